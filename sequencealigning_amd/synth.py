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


# ---- the same generators as torch ops, for batches too large to build on the
# host (configs[2]: 10^6 pairs of 10 kbp); bit-identical to the numpy ones.
def _s64(v: int) -> int:
    return v - (1 << 64) if v >= 1 << 63 else v


_M1, _M2, _GOLD = _s64(0xBF58476D1CE4E5B9), _s64(0x94D049BB133111EB), _s64(0x9E3779B97F4A7C15)


def _shr(z, k: int):
    """Logical right shift of int64 bit patterns."""
    return (z >> k) & ((1 << (64 - k)) - 1)


def splitmix64_torch(seed, idx):
    """splitmix64 output idx + 1 of the stream seeded with `seed` (int64
    tensors or ints, broadcast), as int64 bit patterns."""
    z = seed + (idx + 1) * _GOLD
    z = (z ^ _shr(z, 30)) * _M1
    z = (z ^ _shr(z, 27)) * _M2
    return z ^ _shr(z, 31)


def mut_pairs_torch(n_pairs: int, length: int, delta: float, seed: int, device,
                    chunk: int = 8192):
    """configs[2]-style G-mut batch on `device`: query k = bases
    [k*length, (k+1)*length) of random_bases(seed, n_pairs*length), db k =
    mutate(query k, delta, seed=k) (tools/bench_wfa.py's pairs, every pair
    distinct).  Returns (q_seq, q_off, db_seq, db_off): uint8 device tensors
    and uint64 host offsets, equal to the numpy generators'."""
    import torch
    dev = torch.device(device)
    bases = torch.tensor(list(b"ACGT"), dtype=torch.uint8, device=dev)
    q_seq = torch.empty(n_pairs * length, dtype=torch.uint8, device=dev)
    d_parts, d_lens = [], []
    thr = float(delta)
    for p0 in range(0, n_pairs, chunk):
        p1 = min(n_pairs, p0 + chunk)
        P = p1 - p0
        idx = torch.arange(p0 * length, p1 * length, dtype=torch.int64, device=dev)
        q = bases[_shr(splitmix64_torch(seed, idx), 62)].view(P, length)
        q_seq[p0 * length:p1 * length] = q.reshape(-1)
        # mutate(q_k, delta, seed=k): one stream of 3*length outputs per pair
        ks = torch.arange(p0, p1, dtype=torch.int64, device=dev).view(P, 1)
        j = torch.arange(length, dtype=torch.int64, device=dev).view(1, length)
        u = _shr(splitmix64_torch(ks, j), 11).to(torch.float64) / float(1 << 53)
        ev = _shr(splitmix64_torch(ks, j + length), 62)
        rb = _shr(splitmix64_torch(ks, j + 2 * length), 60)
        del j
        hit = u < thr
        del u
        sub = hit & (ev <= 1)
        ins = hit & (ev == 2)
        dele = hit & (ev == 3)
        del ev, hit
        code = torch.searchsorted(bases, q.contiguous())
        base = torch.where(sub, bases[(code + 1 + (rb % 3)) % 4], q)
        del code, sub
        cnt = torch.ones((P, length), dtype=torch.int64, device=dev)
        cnt[ins] = 2
        cnt[dele] = 0
        row_len = cnt.sum(1)
        csum = torch.cumsum(cnt, 1)
        start = csum - cnt                                  # position within the row
        row_off = torch.cumsum(row_len, 0) - row_len        # row start within the chunk
        pos = start + row_off.view(P, 1)
        out = torch.empty(int(row_len.sum()), dtype=torch.uint8, device=dev)
        keep = cnt > 0
        out[pos[keep]] = base[keep]
        out[pos[ins] + 1] = bases[rb[ins] & 3]
        d_parts.append(out)
        d_lens.append(row_len.cpu())
        del cnt, csum, start, pos, keep, ins, dele, rb, base, q
    d_seq = torch.cat(d_parts) if d_parts else torch.empty(0, dtype=torch.uint8, device=dev)
    lens = torch.cat(d_lens).numpy() if d_lens else np.zeros(0, np.int64)
    q_off = np.arange(n_pairs + 1, dtype=np.uint64) * np.uint64(length)
    d_off = np.zeros(n_pairs + 1, np.uint64)
    d_off[1:] = np.cumsum(lens)
    return q_seq, q_off, d_seq, d_off
