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

``ShardedAllVsAll`` is the configs[4] (C5) driver: score-only all-vs-all with
the db sharded over the ranks (``saln_nw_avsa_*`` per rank on its own GPU)
and the 8-byte {score, status} records gathered to rank 0 in the reference's
db-outer / query-inner order with one RCCL gather.
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
    from .nw import CigarBatch, nw_align_batch
    world, rank = dist.get_world_size(), dist.get_rank()
    dev = torch.cuda.current_device() if device is None else device
    lo, hi = shard_db([len(d) for d in dbs], world, rank)
    res, cigs = nw_align_batch(queries, dbs[lo:hi], scoring=scoring, device=dev)
    backend = dist.get_backend()
    tdev = torch.device("cuda", dev) if backend == "nccl" else torch.device("cpu")
    rec = torch.from_numpy(res.view(np.int32).copy()).to(tdev)
    allrec = gather_records(rec)
    # CIGARs: lengths, then the words (the engine's length << 4 | op), through
    # the same gather
    lens_np = np.asarray(res["cigar_len"], np.int64)
    flat = (np.concatenate([cigs.words(k) for k in range(len(cigs))]).astype(np.int64)
            if len(cigs) else np.zeros(0, np.int64))
    lens = torch.from_numpy(lens_np).to(tdev)
    cw = torch.from_numpy(flat).to(tdev)
    all_lens = gather_records(lens)
    all_words = gather_records(cw)
    if rank != 0:
        return None, None
    out = allrec.cpu().numpy().astype(np.int32).view(_lib.RESULT_DTYPE)
    n_all = all_lens.cpu().numpy().astype(np.int64)
    off = np.zeros(len(n_all), np.int64)
    if len(n_all) > 1:
        off[1:] = np.cumsum(n_all)[:-1]
    return out, CigarBatch(all_words.cpu().numpy().astype(np.uint32), off, n_all)


def shard_counts(db_lengths, world: int) -> list[tuple[int, int]]:
    """[start, end) db block of every rank (``shard_db`` for each rank): any
    rank can size every other rank's block without communicating."""
    return [shard_db(db_lengths, world, r) for r in range(world)]


def _avsa_engine(device: int, scoring=None):
    """Default per-rank engine of ShardedAllVsAll: libsaln's score-only
    all-vs-all (NwAllVsAll) on `device`, sequences resident in HBM."""
    import torch

    from .nw import NwAllVsAll

    class _Engine:
        def __init__(self, q_seq, q_off, d_seq, d_off):
            dev = torch.device("cuda", device)
            self.av = NwAllVsAll(q_off, d_off, scoring=scoring, device=device)
            self.cells = self.av.cells
            self.q = torch.from_numpy(np.ascontiguousarray(q_seq, np.uint8)).to(dev)
            self.d = torch.from_numpy(np.ascontiguousarray(d_seq, np.uint8)).to(dev)
            if self.q.numel() == 0:
                self.q = torch.zeros(1, dtype=torch.uint8, device=dev)
            if self.d.numel() == 0:
                self.d = torch.zeros(1, dtype=torch.uint8, device=dev)

        def __call__(self, out):
            if out.numel():
                self.av.execute(self.q, self.d, out)

        def status(self) -> int:
            """Device error flags of the executes since the last call (blocks)."""
            import ctypes as C

            from . import _lib
            f = C.c_uint32()
            rc = _lib.lib().saln_nw_avsa_status(self.av._h, C.byref(f))
            if rc not in (_lib.OK, _lib.E_DEVICE_WAIT):
                _lib.check(rc, "saln_nw_avsa_status")
            return f.value

        def close(self):
            self.av.close()

    return _Engine


class ShardedAllVsAll:
    """configs[4]: every (db d, query q) pair of the reference loop
    (src/main.rs:61-67), score + panic status, with the db sharded over the
    ranks of the default process group (contiguous blocks balanced by
    cumulative length; queries replicated).  ``execute`` runs this rank's
    block and gathers all blocks to rank 0 with one ``dist.gather`` of
    equal-sized int32 buffers (RCCL over xGMI with the nccl backend, host
    tensors with gloo).  Rank blocks are contiguous in the reference's pair
    order, so the gathered buffer is the reference's db-outer / query-inner
    order: ``result()`` on rank 0 returns (scores, statuses) int32[n_db, n_q].

    ``engine`` (tests) replaces the per-rank compute: a class built as
    engine(q_seq, q_off, d_seq, d_off) with ``cells``, ``__call__(out)`` that
    fills out (int32[n_block_db * n_q * 2], on the engine's device),
    ``close()`` and optionally ``status()`` (device error flags since the
    last call, include/saln.h saln_nw_avsa_status).

    ``execute`` checks the device status of every rank's block before the
    gather (a MAX all-reduce of one flag word): a rank whose column-stripe
    fill timed out makes every rank raise instead of gathering wrong
    records, or hanging in the gather."""

    def __init__(self, q_seq, q_off, db_seq, db_off, *, scoring=None, device: int | None = None,
                 engine=None, dst: int = 0):
        import torch
        import torch.distributed as dist
        self.pg = dist.is_available() and dist.is_initialized()
        # without a process group: one rank, the gather is a no-op
        self.world, self.rank = (dist.get_world_size(), dist.get_rank()) if self.pg else (1, 0)
        self.dst = dst
        q_off = np.ascontiguousarray(q_off, np.uint64)
        db_off = np.ascontiguousarray(db_off, np.uint64)
        self.n_q, self.n_db = len(q_off) - 1, len(db_off) - 1
        lens = (db_off[1:] - db_off[:-1]).astype(np.int64)
        self.blocks = shard_counts(lens, self.world)
        lo, hi = self.blocks[self.rank]
        self.lo, self.hi = lo, hi
        d0, d1 = int(db_off[lo]), int(db_off[hi])
        sub_off = db_off[lo:hi + 1] - np.uint64(d0)
        sub_seq = np.asarray(db_seq, np.uint8)[d0:d1]
        if engine is None:
            dev = torch.cuda.current_device() if device is None else device
            engine = _avsa_engine(dev, scoring)
            self.dev = torch.device("cuda", dev)
        else:
            self.dev = torch.device("cpu")
        self.engine = engine(np.asarray(q_seq, np.uint8), q_off, sub_seq, sub_off)
        self.cells_local = int(self.engine.cells)
        self.cells_total = int(q_off[-1]) * int(db_off[-1])
        self.counts = [(b - a) * self.n_q * 2 for a, b in self.blocks]
        self.cap = max(1, max(self.counts))
        # this rank's records at the head of a cap-sized buffer (the gather
        # needs equal sizes); the engine writes into it directly
        self.local = torch.zeros(self.cap, dtype=torch.int32, device=self.dev)
        self.comm_dev = (self.dev if not self.pg or dist.get_backend() == "nccl"
                         else torch.device("cpu"))
        self.parts = None
        if not self.pg:
            self.big = self.local
            self.parts = [self.local]
        elif self.rank == dst:
            self.big = torch.zeros(self.world * self.cap, dtype=torch.int32, device=self.comm_dev)
            self.parts = list(self.big.view(self.world, self.cap).unbind(0))

    @property
    def cells(self) -> int:
        """Cells of all ranks (sum over pairs of len_q * len_db)."""
        return self.cells_total

    def execute(self, gather: bool = True, check: bool = True) -> None:
        self.engine(self.local[:self.counts[self.rank]])
        if check:
            self.check()
        if gather:
            self.gather()

    def check(self) -> None:
        """Raise on every rank if any rank's engine reported a device error
        (SALN_E_DEVICE_WAIT) since the last check."""
        import torch
        import torch.distributed as dist

        from . import _lib
        status = getattr(self.engine, "status", None)
        flags = int(status()) if status is not None else 0
        if self.pg:
            t = torch.tensor([flags], dtype=torch.int64, device=self.comm_dev)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            flags = int(t.item())
        if flags:
            raise _lib.SalnError(_lib.E_DEVICE_WAIT,
                                 f"ShardedAllVsAll execute: device flags {flags:#x} on some rank "
                                 "(a column-stripe dependency wait timed out)")

    def gather(self) -> None:
        import torch.distributed as dist
        if not self.pg:
            return
        src = self.local if self.comm_dev == self.dev else self.local.to(self.comm_dev)
        dist.gather(src, self.parts, dst=self.dst)

    def result(self):
        """(scores, statuses) int32[n_db, n_q] in the reference order on the
        gathering rank, None elsewhere (after execute)."""
        if self.rank != self.dst:
            return None
        big = self.big.view(self.world, self.cap).cpu().numpy()
        flat = np.concatenate([big[r, :c] for r, c in enumerate(self.counts)])
        h = flat.reshape(self.n_db, self.n_q, 2)
        return h[..., 0].copy(), h[..., 1].copy()

    def lookup(self, d_idx, q_idx):
        """(scores, statuses) of pairs (db d_idx[k], query q_idx[k]) read from
        the gathered buffer on the gathering rank (no full host copy)."""
        import torch
        d_idx = np.asarray(d_idx, np.int64)
        q_idx = np.asarray(q_idx, np.int64)
        starts = np.array([a for a, _ in self.blocks], np.int64)
        r = np.searchsorted(starts, d_idx, side="right") - 1
        while True:  # empty blocks share a start: step to the rank that holds d
            hi = np.array([self.blocks[x][1] for x in r])
            over = d_idx >= hi
            if not over.any():
                break
            r[over] += 1
        pos = r * self.cap + (d_idx - starts[r]) * self.n_q * 2 + q_idx * 2
        t = torch.from_numpy(pos).to(self.big.device)
        return self.big[t].cpu().numpy(), self.big[t + 1].cpu().numpy()

    def status_count(self, status: int) -> int:
        """Number of gathered pairs with this status (gathering rank)."""
        n = 0
        for r, c in enumerate(self.counts):
            n += int((self.parts[r][1:c:2] == status).sum())
        return n

    def close(self) -> None:
        self.engine.close()


def nw_score_all_vs_all_sharded(queries, dbs, *, scoring=None, device: int | None = None,
                                engine=None):
    """Host-sequence front end of ShardedAllVsAll: (scores, statuses) on
    rank 0 (int32[n_db, n_q], reference order), None elsewhere."""
    from .nw import pack_csr
    q_seq, q_off = pack_csr(queries)
    d_seq, d_off = pack_csr(dbs)
    s = ShardedAllVsAll(q_seq, q_off, d_seq, d_off, scoring=scoring, device=device,
                        engine=engine)
    s.execute()
    out = s.result()
    s.close()
    return out
