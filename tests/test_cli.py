"""CPU: the `saln` CLI's argument handling and the input errors it reports
before it touches a GPU (main.rs:19-60, parse.rs:8-50): help, unknown and
missing arguments (clap-style exit 2), an unreadable FASTA (the reference
prints and returns 0), and `-a a-star`, which this engine does not provide."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "sequencealigning_amd", "saln")

pytestmark = pytest.mark.skipif(not os.path.exists(CLI), reason="CLI not built")


def _run(*args):
    return subprocess.run([CLI, *args], capture_output=True, text=True, timeout=60)


def test_help_lists_the_reference_flags():
    r = _run("--help")
    assert r.returncode == 0
    for flag in ("--query-file", "--db-file", "--out-path", "--verbose", "--mode", "--algo",
                 "--stage-times", "--max-blocks"):
        assert flag in r.stdout, flag


def test_unknown_and_missing_arguments_exit_2():
    r = _run("--bogus")
    assert r.returncode == 2 and "unexpected argument '--bogus'" in r.stderr
    r = _run("-q", "x.fa")
    assert r.returncode == 2 and "--db-file" in r.stderr
    r = _run("-q", "x.fa", "-d", "y.fa", "-m", "sideways")
    assert r.returncode == 2 and "invalid value 'sideways'" in r.stderr


def test_option_flag_is_checked_before_any_work(tmp_path):
    """--option NAME=VALUE goes to saln_option_set before the context exists:
    a malformed pair is a usage error, an unknown name or an out-of-range
    value stops the run with exit 2 (no GPU needed for either)."""
    fa = tmp_path / "a.fa"
    fa.write_text(">a\nACGT\n")
    base = ("-q", str(fa), "-d", str(fa), "-a", "needleman-wunsch")
    r = _run(*base, "--option", "host.prefault_mb")
    assert r.returncode == 2 and "invalid value 'host.prefault_mb'" in r.stderr
    r = _run(*base, "--option=host.prefault_mb=x")
    assert r.returncode == 2 and "invalid value" in r.stderr
    r = _run(*base, "--option", "nw.no_such_knob=1")
    assert r.returncode == 2 and "--option nw.no_such_knob=1" in r.stderr
    r = _run(*base, "--option", "nw.pk_tab=9")
    assert r.returncode == 2 and "--option nw.pk_tab=9" in r.stderr
    assert "--option <NAME=VALUE>" in _run("--help").stdout


def test_unreadable_fasta_is_reported_and_returns(tmp_path):
    good = tmp_path / "d.fa"
    good.write_text(">d\nACGT\n")
    r = _run("-q", str(tmp_path / "missing.fa"), "-d", str(good), "-a", "needleman-wunsch")
    assert r.returncode == 0
    assert "Query fasta could not be opened" in r.stderr and "aborting" in r.stderr


def test_a_star_is_rejected(tmp_path):
    f = tmp_path / "q.fa"
    f.write_text(">q\nACGT\n")
    r = _run("-q", str(f), "-d", str(f))  # the reference's default algorithm
    assert r.returncode == 2 and "a-star" in r.stderr
