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


def test_render_batch_matches_oracle(saln, oracle):
    """saln_nw_render_batch (every pair computed once, one plan) gives the
    oracle's literal-DFS text for every pair of an all-vs-all batch with
    empty, short, tie-heavy and panicking pairs; stop_at_panic ends the list
    at the first panicking pair, as the reference's abort does."""
    import numpy as np
    from nw_check import rand_seq
    rng = np.random.default_rng(77)
    queries = [b"", b"A", b"TA", b"AAA"] + [rand_seq(rng, int(n)) for n in (5, 9, 17, 30)] + \
        [bytes(rng.choice([65, 67], 10).astype(np.uint8))]
    dbs = [b"", b"A", b"AA"] + [rand_seq(rng, int(n)) for n in (6, 13, 28)] + \
        [bytes(rng.choice([65, 67], 11).astype(np.uint8))]
    out = saln.render_batch(queries, dbs)
    assert len(out) == len(queries) * len(dbs)
    k = 0
    for d in dbs:
        for q in queries:
            o = oracle.nw(q, d)
            text, blocks, status = out[k]
            assert o.dfs_rc in (0, 1), (q, d)
            assert text == o.stdout, (q, d)
            assert blocks == o.dfs_blocks and (status == 2) == (o.dfs_rc == 1), (q, d)
            k += 1
    first = next(k for k, (_, _, s) in enumerate(out) if s == 2)
    assert saln.render_batch(queries, dbs, stop_at_panic=True) == out[:first + 1]
    # the single-pair form is the same call
    assert saln.render(queries[7], dbs[5]) == out[5 * len(queries) + 7]


@pytest.mark.parametrize("chunk", [None, 1, 4])
def test_cli_nw_aborts_at_first_panic(tmp_path, chunk):
    """Without --no-abort the CLI stops at the first pair whose traceback
    panics (N5: TA vs A), after the text of the pairs before it, with the
    reference's exit code 101; later pairs print nothing - also when the
    pairs before it were printed by the printer thread of an earlier chunk."""
    _fasta(tmp_path / "q.fa", [("q1", "GATTACA"), ("q2", "TA"), ("q3", "ACGT")])
    _fasta(tmp_path / "d.fa", [("d1", "A"), ("d2", "GATTACA")])
    p = subprocess.run([CLI, "-q", str(tmp_path / "q.fa"), "-d", str(tmp_path / "d.fa"),
                        "-a", "needleman-wunsch", "--no-timing"]
                       + (["--chunk-pairs", str(chunk)] if chunk else []),
                       capture_output=True, timeout=120)
    assert p.returncode == 101, p.stderr
    assert b"panicked" in p.stderr
    import sequencealigning_amd as saln
    want = saln.render(b"GATTACA", b"A")[0] + saln.render(b"TA", b"A")[0]
    assert p.stdout.decode() == want


@pytest.mark.parametrize("chunk", [None, 7, 64])
def test_cli_nw_batch_max_blocks_matches_oracle(tmp_path, oracle, chunk):
    """A C2-shaped run through the batched CLI (24 x 24 records of 150 bp):
    with --max-blocks 1 --no-abort every pair's text is the oracle's literal
    DFS stopped before its second block, in the reference's order - also in
    chunks of 7 and 64 pairs (the first a quarter of that), each printed on a
    thread while the next renders."""
    from sequencealigning_amd import synth
    n, L = 24, 150
    qs, qo, ds, do = synth.iid_pairs(n, L, L, seed=0x5EED0002)
    q = [qs[int(qo[k]):int(qo[k + 1])].tobytes().decode() for k in range(n)]
    d = [ds[int(do[k]):int(do[k + 1])].tobytes().decode() for k in range(n)]
    _fasta(tmp_path / "q.fa", [(f"q{k}", s) for k, s in enumerate(q)])
    _fasta(tmp_path / "d.fa", [(f"d{k}", s) for k, s in enumerate(d)])
    p = subprocess.run([CLI, "-q", str(tmp_path / "q.fa"), "-d", str(tmp_path / "d.fa"),
                        "-a", "needleman-wunsch", "--no-timing", "--no-abort", "--max-blocks", "1"]
                       + (["--chunk-pairs", str(chunk)] if chunk else []),
                       capture_output=True, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    want = "".join(oracle.nw(a.encode(), b.encode(), max_blocks=1, max_pops=10**8).stdout
                   for b in d for a in q)
    assert p.stdout.decode() == want


@pytest.mark.parametrize("max_blocks", [1, 2, 50, 0])
def test_render_batch_gpu_decided_matches_oracle(saln, oracle, max_blocks):
    """Render batches decide most pairs on the GPU (the first walk and the
    DFS's next event, nw_next_event_kernel) and run the host DFS only for
    the rest; every pair's text, block count and status equal the oracle's
    literal DFS (stopped at max_blocks) on configs[1]-shaped i.i.d. pairs,
    5 % mutated pairs (co-optimal gap placements), two-letter pairs (many
    co-optimal paths), N, '-' bytes (a bar where a '-' meets a gap, as in the
    reference's Display) and panicking pairs.  All blocks (max_blocks 0) only
    on the mutated pairs: an i.i.d. pair can have millions of co-optimal
    alignments, past the oracle's text buffer."""
    import numpy as np
    from nw_check import rand_seq

    from sequencealigning_amd import synth
    rng = np.random.default_rng(303 + max_blocks)
    qs, ds = [], []
    for k in range(120):
        q = rand_seq(rng, int(rng.integers(100, 160)))
        kind = k % 4 if max_blocks else 1 + 2 * (k % 2)
        if kind == 0:
            d = rand_seq(rng, int(rng.integers(100, 160)))
        elif kind == 1:
            d = synth.mutate(q, 0.05, seed=k)
        elif kind == 2:
            q = bytes(rng.choice([65, 67], len(q)).astype(np.uint8))
            d = bytes(rng.choice([65, 67], int(rng.integers(90, 150))).astype(np.uint8))
        else:
            d = synth.mutate(q, 0.1, seed=k)[:int(rng.integers(60, 140))]
        qs.append(q)
        ds.append(d)
    qs += [b"TA", b"NNACGTN", b"AAA", b"", b"AC-GTA-", b"--"]
    ds += [b"A", b"ACGGT", b"AA", b"", b"A-CGTA", b"-"]
    n = len(qs)
    st = {}
    out = saln.render_batch(qs, ds, pairs=[(k, k) for k in range(n)], max_blocks=max_blocks,
                            stats=st)
    assert len(out) == n
    for k in range(n):
        o = oracle.nw(qs[k], ds[k], max_blocks=max_blocks, max_pops=10**8, out_cap=1 << 26)
        text, blocks, status = out[k]
        assert len(o.stdout) < (1 << 26), k
        assert o.dfs_rc in (0, 1, 3), (k, o.dfs_rc)
        assert text == o.stdout, k
        assert blocks == o.dfs_blocks, k
        want = {0: saln._lib.OK, 1: saln._lib.REF_PANIC_BOUNDARY, 3: saln._lib.ENUM_CAP}[o.dfs_rc]
        assert status == want, (k, status, o.dfs_rc)
    # the GPU settles every sentinel-free pair under max_blocks = 1, and the
    # pairs with one co-optimal alignment (or none printed) otherwise
    assert st["gpu_decided"] >= (n - 10 if max_blocks == 1 else 1), st
