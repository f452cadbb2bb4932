"""Deterministic synthetic DNA: splitmix64 in counter form,
i.i.d. uniform ACGT.  G-iid: query and db drawn independently.  G-mut(delta):
db = query mutated per base with probability delta (substitution 1/2 to a
different base, insertion 1/4 of one random base after it, deletion 1/4)."""
from __future__ import annotations

import numpy as np

BASES = np.frombuffer(b"ACGT", np.uint8)
_GOLDEN = np.uint64(0x9E3779B97F4A7C15)


def splitmix64(seed: int, n: int, start: int = 0) -> np.ndarray:
    """Outputs start..start+n-1 of the splitmix64 stream seeded with `seed`."""
    with np.errstate(over="ignore"):
        z = np.uint64(seed) + (np.arange(start + 1, start + n + 1, dtype=np.uint64) * _GOLDEN)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def random_bases(seed: int, n: int, start: int = 0) -> np.ndarray:
    return BASES[(splitmix64(seed, n, start) >> np.uint64(62)).astype(np.intp)]


def iid_pairs(n_pairs: int, len_q: int, len_db: int, seed: int):
    """G-iid batch as CSR arrays: (q_seq, q_off, db_seq, db_off), pair k = (k, k)."""
    q = random_bases(seed, n_pairs * len_q)
    d = random_bases(seed ^ 0xD5D5D5D5, n_pairs * len_db)
    q_off = np.arange(n_pairs + 1, dtype=np.uint64) * np.uint64(len_q)
    d_off = np.arange(n_pairs + 1, dtype=np.uint64) * np.uint64(len_db)
    return q, q_off, d, d_off


def mutate(seq: bytes | np.ndarray, delta: float, seed: int) -> bytes:
    s = np.frombuffer(bytes(seq), np.uint8)
    n = len(s)
    if n == 0:
        return b""
    r = splitmix64(seed, 3 * n)
    u = (r[:n] >> np.uint64(11)).astype(np.float64) / float(1 << 53)
    ev = (r[n:2 * n] >> np.uint64(62)).astype(np.int64)      # 0,1 sub; 2 ins; 3 del
    rb = (r[2 * n:] >> np.uint64(60)).astype(np.int64)
    code = np.searchsorted(BASES, s)
    hit = u < delta
    sub = hit & (ev <= 1)                                   # substitution to a different base
    ins = hit & (ev == 2)                                   # insertion after the base
    dele = hit & (ev == 3)                                  # deletion
    base = s.copy()
    base[sub] = BASES[(code[sub] + 1 + (rb[sub] % 3)) % 4]
    cnt = np.ones(n, np.int64)
    cnt[ins] = 2
    cnt[dele] = 0
    out = np.repeat(base, cnt)
    start = np.cumsum(cnt) - cnt
    out[start[ins] + 1] = BASES[rb[ins] & 3]
    return out.tobytes()


def mut_pair(length: int, delta: float, seed: int) -> tuple[bytes, bytes]:
    q = random_bases(seed, length).tobytes()
    return q, mutate(q, delta, seed ^ 0x5A5A5A5A)
