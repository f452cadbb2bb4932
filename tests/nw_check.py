"""Shared helpers for NW parity tests (imports the oracle: test-only)."""
from __future__ import annotations

import numpy as np

SCHEME = (5, -4, -8, -6)


def rand_seq(rng: np.random.Generator, n: int, alphabet: bytes = b"ACGT") -> bytes:
    a = np.frombuffer(alphabet, np.uint8)
    return a[rng.integers(0, len(a), n)].tobytes()


def path_score(query: bytes, db: bytes, cigar, scheme=SCHEME) -> tuple[int, bool]:
    """Score of an alignment path under the reference recurrences (I/D open
    only from M, needleman_wunsch_affine.rs:87-94); second value is False if
    the path breaks a recurrence rule or does not consume both sequences."""
    mat, mis, go, ge = scheme
    i = j = 0
    state = "M"
    score = 0
    ok = True
    for n, op in cigar:
        for _ in range(n):
            if op in "=X":
                if j >= len(query) or i >= len(db):
                    return score, False
                eq = query[j] == db[i]
                if (op == "=") != eq:
                    ok = False
                score += mat if eq else mis
                i += 1; j += 1; state = "M"
            elif op == "I":
                if state == "D" or j >= len(query):
                    ok = False
                score += (go + ge) if state == "M" else ge
                j += 1; state = "I"
            else:
                if state == "I" or i >= len(db):
                    ok = False
                score += (go + ge) if state == "M" else ge
                i += 1; state = "D"
    return score, ok and i == len(db) and j == len(query)


def expand(cigar) -> str:
    return "".join(op * n for n, op in cigar)
