"""Multi-GPU driver for the pair loop.

The reference aligns every query against every db record, db outer / query
inner (src/main.rs:61-62), and the pairs are independent.  One process per
GPU (torch.distributed; backend "nccl" = RCCL over xGMI on MI355X):

* ``shard_db`` splits the db records into contiguous blocks balanced by
  cumulative length, one per rank; queries are replicated;
* each rank runs its block through libsaln on its own GPU;
* ``gather_records`` collects the fixed-size per-pair records on rank 0
  (one gather of equal-sized, padded buffers); concatenating the rank blocks
  in rank order restores the reference's pair order exactly.

No collective sits on the alignment path itself; the gather is the only
exchange.
"""
from __future__ import annotations

import numpy as np


def shard_db(db_lengths, world: int, rank: int) -> tuple[int, int]:
    """Contiguous [start, end) block of db records for `rank`, balanced by
    cumulative length (cells scale with len_db for a fixed query set)."""
    lens = np.asarray(db_lengths, dtype=np.int64)
    n = len(lens)
    if world <= 1 or n == 0:
        return (0, n) if rank == 0 else (n, n)
    cum = np.concatenate([[0], np.cumsum(np.maximum(lens, 1))])
    total = cum[-1]
    cuts = [0]
    for r in range(1, world):
        cuts.append(int(np.searchsorted(cum, total * r / world, side="left")))
    cuts.append(n)
    cuts = np.maximum.accumulate(np.minimum(np.array(cuts), n))
    return int(cuts[rank]), int(cuts[rank + 1])


def gather_records(local, group=None, dst: int = 0):
    """Gather a rank-local 1-D tensor of per-pair records (any dtype, any
    length per rank) to `dst`.  Returns the concatenation in rank order on
    `dst` and None elsewhere.  Works with the nccl (device tensors) and gloo
    (host tensors) backends."""
    import torch
    import torch.distributed as dist
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    n = torch.tensor([local.numel()], dtype=torch.int64, device=local.device)
    sizes = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(sizes, n, group=group)
    sizes = [int(s.item()) for s in sizes]
    cap = max(sizes) if sizes else 0
    buf = torch.zeros(cap, dtype=local.dtype, device=local.device)
    buf[:local.numel()] = local
    parts = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
    dist.gather(buf, parts, dst=dst, group=group)
    if rank != dst:
        return None
    return torch.cat([p[:s] for p, s in zip(parts, sizes)])


def nw_align_sharded(queries, dbs, *, scoring=None, device: int | None = None):
    """All-vs-all NW (reference order) with the db sharded over the ranks of
    the default process group.  Returns (results structured array, cigars)
    on rank 0, (None, None) elsewhere."""
    import torch
    import torch.distributed as dist

    from . import _lib
    from .nw import nw_align_batch
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = torch.cuda.current_device() if device is None else device
    lo, hi = shard_db([len(d) for d in dbs], world, rank)
    res, cigs = nw_align_batch(queries, dbs[lo:hi], scoring=scoring, device=dev)
    backend = dist.get_backend()
    tdev = torch.device("cuda", dev) if backend == "nccl" else torch.device("cpu")
    rec = torch.from_numpy(res.view(np.int32).copy()).to(tdev)
    allrec = gather_records(rec)
    # CIGARs: lengths, then the words, through the same gather
    flat = [((n << 4) | {"=": 7, "X": 8, "I": 1, "D": 2}[op]) for c in cigs for n, op in c]
    lens = torch.tensor([len(c) for c in cigs], dtype=torch.int64, device=tdev)
    cw = torch.tensor(flat, dtype=torch.int64, device=tdev)
    all_lens = gather_records(lens)
    all_words = gather_records(cw)
    if rank != 0:
        return None, None
    out = allrec.cpu().numpy().astype(np.int32).view(_lib.RESULT_DTYPE)
    cig, pos = [], 0
    words = all_words.cpu().numpy()
    for n in all_lens.cpu().numpy():
        cig.append([(int(w) >> 4, _lib.CIGAR_OPS[int(w) & 15]) for w in words[pos:pos + n]])
        pos += int(n)
    return out, cig
