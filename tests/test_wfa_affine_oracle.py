"""CPU: the corrected-WFA oracle (oracle/refaffine.c, Gotoh DP) against an
exhaustive enumeration of alignments for tiny pairs, and hand-derived
values.  The corrected gap-affine WFA is SURVEY.md §8(f) row 4 — a
separately labelled engine, parity unpinned against the reference (whose
wfa_align has no defined output for such inputs)."""
import functools
import itertools

import numpy as np
import pytest

from oracle import refcpu

X, O, E = 4, 2, 6  # src/wfa.rs:14-21


def brute(q: bytes, d: bytes, x=X, o=O, e=E) -> int:
    """Minimum over every alignment (column strings over {M, I, D}) of
    x * mismatches + sum over maximal I / D runs of o + e * len."""
    best = None

    @functools.lru_cache(maxsize=None)
    def go(i, j, last):
        # i over q, j over d; last: op of the previous column ('M', 'I', 'D', None)
        if i == len(q) and j == len(d):
            return 0
        r = []
        if i < len(q) and j < len(d):
            r.append((0 if q[i] == d[j] else x) + go(i + 1, j + 1, "M"))
        if i < len(q):  # query base vs gap
            r.append((e if last == "Q" else o + e) + go(i + 1, j, "Q"))
        if j < len(d):  # gap vs db base
            r.append((e if last == "T" else o + e) + go(i, j + 1, "T"))
        return min(r)

    best = go(0, 0, None)
    return best


KATS = [
    (b"", b"", 0),
    (b"A", b"", 8),
    (b"", b"ACGT", 26),
    (b"ACGT", b"ACGT", 0),
    (b"ACGT", b"AGGT", 4),
    (b"ACGT", b"ACT", 8),
    (b"AAAA", b"AA", 14),        # one gap of 2: 2 + 12
    (b"ACGTACGT", b"ACGTTACGT", 8),
    (b"AC", b"CA", 8),           # two mismatches (8) ties an I + D pair (16)? no: 8
]


@pytest.mark.parametrize("q,d,want", KATS)
def test_affine_kats(q, d, want):
    assert refcpu.affine_penalty(q, d) == want
    assert brute(q, d) == want


def test_affine_matches_enumeration():
    rng = np.random.default_rng(5)
    for _ in range(300):
        lq, ld = rng.integers(0, 7, 2)
        q = bytes(rng.choice(list(b"ACGT"), lq).astype(np.uint8))
        d = bytes(rng.choice(list(b"ACGT"), ld).astype(np.uint8))
        pen = [(4, 2, 6), (1, 3, 1), (5, 0, 2)][int(rng.integers(0, 3))]
        assert refcpu.affine_penalty(q, d, *pen) == brute(q, d, *pen), (q, d, pen)


def test_affine_run_pairs_matches_single():
    rng = np.random.default_rng(6)
    qs = [bytes(rng.choice(list(b"ACGT"), int(n)).astype(np.uint8)) for n in rng.integers(0, 60, 9)]
    ds = [bytes(rng.choice(list(b"ACGT"), int(n)).astype(np.uint8)) for n in rng.integers(0, 60, 7)]
    qo = np.concatenate([[0], np.cumsum([len(s) for s in qs])]).astype(np.uint64)
    do = np.concatenate([[0], np.cumsum([len(s) for s in ds])]).astype(np.uint64)
    pq, pd = np.array(list(itertools.product(range(9), range(7)))).T
    got = refcpu.affine_run_pairs(np.frombuffer(b"".join(qs) or b"\0", np.uint8), qo,
                                  np.frombuffer(b"".join(ds) or b"\0", np.uint8), do, pq, pd,
                                  threads=3)
    want = [refcpu.affine_penalty(qs[a], ds[b]) for a, b in zip(pq, pd)]
    assert list(got) == want
