"""CPU: the oracle (oracle/refcpu.c) against the hand-derived KATs of
SURVEY.md §8.4 and against itself (literal DFS vs memoised DFS).  These are
the pins of NW parity: the reference's own NW tests are empty stubs
(needleman_wunsch_affine.rs:458-470), so NW parity is pinned by hand KATs,
not by reference-run fixtures."""
import json
import os

import numpy as np
import pytest

from nw_check import path_score, rand_seq

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def test_hand_kats(oracle):
    with open(os.path.join(GOLDEN, "nw_kats.json")) as f:
        data = json.load(f)
    for k in data["hand"]:
        o = oracle.nw(k["query"].encode(), k["db"].encode())
        assert o.score == k["score"], k["id"]
        assert o.stdout == k["stdout"], k["id"]
        assert (o.dfs_rc == 1) == k["panics"], k["id"]
        assert o.panics == k["panics"], k["id"]
    # N4 worked cells (interior, [x][y] 1-based)
    o = oracle.nw(b"AAA", b"AA")
    for st, arr in (("M", o.M), ("I", o.I), ("D", o.D)):
        assert arr[1:, 1:].tolist() == data["n4_cells"][st], st


def test_boundary_quirks(oracle):
    """needleman_wunsch_affine.rs:183-216: D on row 0, I on column 0, one extra
    extension, sentinel i16::MIN."""
    o = oracle.nw(b"ACGT", b"AC", literal_dfs=False)
    assert o.D[0, 1:].tolist() == [-8 - 6 * (j + 1) for j in range(1, 5)]
    assert o.I[1:, 0].tolist() == [-8 - 6 * (i + 1) for i in range(1, 3)]
    assert (o.M[0, 1:] == -32768).all() and (o.M[1:, 0] == -32768).all()
    assert o.I[0, 0] == -32768 and o.D[0, 0] == -32768 and o.M[0, 0] == 0


def test_literal_vs_memoised(oracle):
    rng = np.random.default_rng(3)
    for _ in range(300):
        q = rand_seq(rng, int(rng.integers(0, 12)), b"ACGTN")
        d = rand_seq(rng, int(rng.integers(0, 12)), b"ACGTN")
        o = oracle.nw(q, d)
        assert o.dfs_rc in (0, 1)
        assert (o.dfs_rc == 1) == o.panics, (q, d)
        assert o.dfs_blocks == o.n_blocks, (q, d)
        if o.first_ops is not None:
            first = o.stdout.split("alignment found\n")[1]
            s1 = first.split("\n")[1][6:]
            assert len(s1) == len(o.first_ops)


def test_first_alignment_rescored(oracle):
    rng = np.random.default_rng(4)
    for _ in range(100):
        q = rand_seq(rng, int(rng.integers(1, 60)))
        d = rand_seq(rng, int(rng.integers(1, 60)))
        o = oracle.nw(q, d, literal_dfs=False)
        if o.first_ops is None:
            assert o.panics
            continue
        cig = [(1, c) for c in o.first_ops]
        s, ok = path_score(q, d, cig)
        assert ok and s == o.score


def test_golden_random_consistent(oracle):
    with open(os.path.join(GOLDEN, "nw_random.json")) as f:
        pairs = json.load(f)["pairs"]
    for v in pairs[:64]:
        o = oracle.nw(v["query"].encode(), v["db"].encode(), literal_dfs=False)
        assert o.score == v["score"]
        assert o.first_ops == v["first_ops"]
        assert o.panics == v["panics"]


def test_linear_oracle_matches_full(oracle):
    """reflinear.c (linear memory, column stripes on threads) against the full
    matrices + memoised DFS: score, end states and panic status, on small,
    empty, tie-heavy and multi-stripe (lq > 256) pairs, and past the x+y
    ~ 5,450 line where sentinel cells start to tie."""
    from sequencealigning_amd import synth
    rng = np.random.default_rng(11)
    cases = [(b"", b""), (b"A", b""), (b"", b"ACG"), (b"ACGT", b"ACGT"), (b"AAAA", b"A")]
    for _ in range(120):
        cases.append((rand_seq(rng, int(rng.integers(0, 40)), b"ACGTN"),
                      rand_seq(rng, int(rng.integers(0, 40)), b"AC")))
    for lq, ld in [(700, 300), (300, 700), (1100, 40), (3100, 2600)]:
        cases.append((rand_seq(rng, lq, b"ACGT"), rand_seq(rng, ld, b"ACGT")))
    q, d = synth.mut_pair(900, 0.05, 7)
    cases.append((q, d))
    for q, d in cases:
        o = oracle.nw(q, d, literal_dfs=False)
        for threads in (1, 4):
            got = oracle.nw_score_linear(q, d, threads)
            assert got == (o.score, o.end_states, o.panics), (len(q), len(d), threads)


def test_check_pairs_matches_single_pair_oracle(oracle):
    """refcheck.c (the threaded batch checker used at the configs[1] scale)
    gives the same score, end states, panic status and first printed
    alignment as the single-pair oracle, incl. empty sides and N."""
    from sequencealigning_amd import synth
    rng = np.random.default_rng(17)
    pairs = [(b"", b""), (b"", b"AC"), (b"A", b""), (b"TA", b"A"), (b"AAA", b"AA"),
             (b"NNAN", b"ANNN")]
    for k in range(40):
        lq, ld = int(rng.integers(1, 200)), int(rng.integers(1, 200))
        if k % 2:
            q, d = synth.mut_pair(lq, 0.1, 500 + k)
        else:
            q = synth.random_bases(600 + k, lq).tobytes()
            d = synth.random_bases(700 + k, ld).tobytes()
        pairs.append((q, d))
    qo = np.zeros(len(pairs) + 1, np.uint64)
    do = np.zeros(len(pairs) + 1, np.uint64)
    qo[1:] = np.cumsum([len(q) for q, _ in pairs])
    do[1:] = np.cumsum([len(d) for _, d in pairs])
    got = oracle.check_pairs(b"".join(q for q, _ in pairs), qo, b"".join(d for _, d in pairs), do,
                             threads=3)
    ops = {7: "=", 8: "X", 1: "I", 2: "D"}
    for k, (q, d) in enumerate(pairs):
        o = oracle.nw(q, d, literal_dfs=False)
        w = got.cigar_words(k)
        first = None if w is None else "".join(ops[int(x) & 15] * (int(x) >> 4) for x in w)
        assert (int(got.score[k]), int(got.end_states[k]), bool(got.panics[k]), first) == \
            (o.score, o.end_states, o.panics, o.first_ops), k


def test_linear_first_alignment_matches_full_oracle(oracle):
    """reflinear.c's parent-set fill + literal DFS (the checker for pairs too
    large for three full matrices) gives the full-matrix oracle's score, end
    states, panic status and first printed alignment, tie-heavy alphabets
    and empty sides included."""
    rng = np.random.default_rng(23)
    for k in range(200):
        lq, ld = int(rng.integers(0, 50)), int(rng.integers(0, 50))
        a = np.frombuffer([b"ACGT", b"AC", b"A", b"AAAC"][k % 4], np.uint8)
        q = a[rng.integers(0, len(a), lq)].tobytes()
        d = a[rng.integers(0, len(a), ld)].tobytes()
        o = oracle.nw(q, d, literal_dfs=False)
        sc, es, pan, first, _ = oracle.nw_first_linear(q, d, threads=2)
        assert (sc, es, pan, first) == (o.score, o.end_states, o.panics, o.first_ops), k


def test_deadend_fixtures(oracle):
    """tests/golden/nw_deadend.json: pairs past the sentinel line whose DFS
    meets sentinel-rooted subtrees (nothing printed, panics, and a block
    printed after the DFS left a dead subtree); the linear oracle reproduces
    the committed values (make_deadend.py checked both oracles)."""
    with open(os.path.join(GOLDEN, "nw_deadend.json")) as f:
        pairs = json.load(f)["pairs"]
    assert any(p["dead"] and p["first_ops"] for p in pairs)
    assert any(p["dead"] and p["panics"] for p in pairs)
    for p in pairs:
        sc, es, pan, first, dead = oracle.nw_first_linear(p["query"].encode(), p["db"].encode(),
                                                          threads=2)
        assert (sc, es, pan, first, dead) == (p["score"], p["end_states"], p["panics"],
                                              p["first_ops"], p["dead"]), p["id"]
