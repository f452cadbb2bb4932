"""The `saln` CLI as a drop-in for the reference binary (src/main.rs): FASTA
in, the reference's stdout out, for -a needleman-wunsch and -a wfa, checked
against the oracle's text for every pair in db-outer / query-inner order."""
import os
import subprocess

import pytest

pytestmark = pytest.mark.gpu

CLI = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                   "sequencealigning_amd", "saln")


def _fasta(path, recs):
    with open(path, "w") as f:
        for name, seq in recs:
            f.write(f">{name}\n{seq}\n")


def test_cli_nw_matches_oracle(tmp_path, oracle):
    qs = [("q1", "GATTACA"), ("q2", "ACGTTGCA")]
    ds = [("d1", "GATACA"), ("d2", "ACGTGCA"), ("d3", "GGATTACAA")]
    _fasta(tmp_path / "q.fa", qs)
    _fasta(tmp_path / "d.fa", ds)
    p = subprocess.run([CLI, "-q", str(tmp_path / "q.fa"), "-d", str(tmp_path / "d.fa"),
                        "-a", "needleman-wunsch", "--no-timing", "--no-abort"],
                       capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr
    want = "".join(oracle.nw(q.encode(), d.encode()).stdout for _, d in ds for _, q in qs)
    assert p.stdout.decode() == want


def test_cli_wfa_matches_oracle(tmp_path, oracle):
    qs = [("q1", "AC"), ("q2", "GATTACA")]
    ds = [("d1", "AG"), ("d2", "GCATTAC")]
    _fasta(tmp_path / "q.fa", qs)
    _fasta(tmp_path / "d.fa", ds)
    p = subprocess.run([CLI, "-q", str(tmp_path / "q.fa"), "-d", str(tmp_path / "d.fa"),
                        "-a", "wfa", "--no-abort"], capture_output=True, timeout=120)
    assert p.returncode == 0, p.stderr
    want = "".join(oracle.wfa(q.encode(), d.encode(), max_steps=64).stdout
                   for _, d in ds for _, q in qs)
    assert p.stdout.decode() == want


def test_cli_wfa_panic_exit_101(tmp_path):
    from sequencealigning_amd import synth
    q = synth.random_bases(3, 500).tobytes().decode()
    d = synth.mutate(q.encode(), 0.05, seed=4).decode()
    _fasta(tmp_path / "q.fa", [("q", q)])
    _fasta(tmp_path / "d.fa", [("d", d)])
    p = subprocess.run([CLI, "-q", str(tmp_path / "q.fa"), "-d", str(tmp_path / "d.fa"),
                        "-a", "wfa"], capture_output=True, timeout=120)
    assert p.returncode == 101
    assert p.stdout.decode().count("lo: ") == 7
