"""Multi-rank path on CPU with gloo, world_size 2: db
sharding and the rank-0 gather restore the reference's all-vs-all pair order
(db outer, query inner; src/main.rs:61-62)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from sequencealigning_amd.dist import shard_db


def test_shard_db_balanced_and_contiguous():
    rng = np.random.default_rng(0)
    lens = rng.integers(1, 1000, 101)
    for world in (1, 2, 3, 4, 8):
        blocks = [shard_db(lens, world, r) for r in range(world)]
        assert blocks[0][0] == 0 and blocks[-1][1] == len(lens)
        for a, b in zip(blocks, blocks[1:]):
            assert a[1] == b[0]
        loads = [lens[s:e].sum() for s, e in blocks]
        assert max(loads) <= lens.sum() / world + lens.max()
    assert shard_db([], 2, 0) == (0, 0) and shard_db([], 2, 1) == (0, 0)
    assert shard_db([5, 5], 4, 3) == (2, 2)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, n_q, db_lens, out):
    import torch
    import torch.distributed as dist

    from sequencealigning_amd.dist import gather_records, shard_db
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = shard_db(db_lens, world, rank)
    # stand-in per-pair record: (global pair id, rank) for pairs d*n_q + q of my block
    pid = [d * n_q + q for d in range(lo, hi) for q in range(n_q)]
    rec = torch.tensor([v for p in pid for v in (p, rank)], dtype=torch.int32)
    allrec = gather_records(rec)
    if rank == 0:
        out.put(allrec.numpy().reshape(-1, 2).tolist())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gather_restores_reference_order(world):
    n_q = 3
    db_lens = [150, 10, 900, 40, 40, 300, 7]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n_q, db_lens, q))
             for r in range(world)]
    for p in procs:
        p.start()
    got = q.get(timeout=120)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert [g[0] for g in got] == list(range(n_q * len(db_lens)))
    ranks = [g[1] for g in got]
    assert ranks == sorted(ranks) and set(ranks) == set(range(world))


def _gpu_worker(rank, world, port, queries, dbs, out):
    import torch
    import torch.distributed as dist

    from sequencealigning_amd.dist import nw_align_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    res, cig = nw_align_sharded(queries, dbs, device=0)
    if rank == 0:
        out.put((res.tolist(), cig))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_nw_matches_single_process():
    """Two ranks (gloo gather; both on cuda:0 of the box) give the same
    all-vs-all records and CIGARs, in the same order, as one batch."""
    import sequencealigning_amd as saln
    from nw_check import rand_seq
    rng = np.random.default_rng(3)
    queries = [rand_seq(rng, int(rng.integers(20, 200))) for _ in range(5)]
    dbs = [rand_seq(rng, int(rng.integers(20, 200))) for _ in range(9)]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(r, 2, port, queries, dbs, q)) for r in range(2)]
    for p in procs:
        p.start()
    res, cig = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want, want_cig = saln.nw_align_batch(queries, dbs)
    assert res == want.tolist()
    assert cig == want_cig


class _OracleAvsaEngine:
    """CPU stand-in for the per-rank GPU engine of ShardedAllVsAll: the
    oracle's score + panic status of every (db, query) pair of the block, in
    db-outer / query-inner order (test-only)."""

    def __init__(self, q_seq, q_off, d_seq, d_off):
        from oracle import refcpu
        nq, nd = len(q_off) - 1, len(d_off) - 1
        qs = [bytes(q_seq[int(q_off[k]):int(q_off[k + 1])]) for k in range(nq)]
        ds = [bytes(d_seq[int(d_off[k]):int(d_off[k + 1])]) for k in range(nd)]
        pq = [q for _ in ds for q in qs]
        pd = [d for d in ds for _ in qs]
        qo = np.zeros(len(pq) + 1, np.uint64); qo[1:] = np.cumsum([len(x) for x in pq])
        do = np.zeros(len(pd) + 1, np.uint64); do[1:] = np.cumsum([len(x) for x in pd])
        self.want = refcpu.check_pairs(b"".join(pq), qo, b"".join(pd), do, threads=2) \
            if pq else None
        self.cells = sum(len(q) * len(d) for q, d in zip(pq, pd))

    def __call__(self, out):
        import torch
        if self.want is None:
            return
        rec = np.stack([self.want.score, np.where(self.want.panics, 2, 0).astype(np.int32)], 1)
        out.copy_(torch.from_numpy(rec.reshape(-1)))

    def close(self):
        pass


def _avsa_worker(rank, world, port, queries, dbs, out):
    import torch.distributed as dist

    from sequencealigning_amd.dist import nw_score_all_vs_all_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    got = nw_score_all_vs_all_sharded(queries, dbs, engine=_OracleAvsaEngine)
    if rank == 0:
        out.put((got[0].tolist(), got[1].tolist()))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_sharded_all_vs_all_gather(world):
    """configs[4] driver (ShardedAllVsAll) with gloo: db blocks per rank, the
    records gathered to rank 0 equal the single-process all-vs-all (score +
    panic status per (db, query), reference order), incl. empty records and
    unequal blocks."""
    from nw_check import rand_seq
    from oracle import refcpu
    rng = np.random.default_rng(8)
    queries = [rand_seq(rng, int(n)) for n in [0, 3, 40, 150, 151, 90]]
    dbs = [rand_seq(rng, int(n)) for n in [120, 0, 7, 150, 33, 200, 1, 64, 149]]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_avsa_worker, args=(r, world, port, queries, dbs, q))
             for r in range(world)]
    for p in procs:
        p.start()
    scores, status = q.get(timeout=180)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert np.asarray(scores).shape == (len(dbs), len(queries))
    for di, d in enumerate(dbs):
        for qi, qq in enumerate(queries):
            o = refcpu.nw(qq, d, literal_dfs=False)
            assert scores[di][qi] == o.score, (di, qi)
            assert (status[di][qi] == 2) == o.panics, (di, qi)


def _avsa_gpu_worker(rank, world, port, queries, dbs, out):
    import torch
    import torch.distributed as dist

    from sequencealigning_amd.dist import nw_score_all_vs_all_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    got = nw_score_all_vs_all_sharded(queries, dbs, device=0)
    if rank == 0:
        out.put((got[0], got[1]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_all_vs_all_gpu_matches_single_process():
    """Two ranks (gloo gather; both on cuda:0 of the box) running libsaln's
    score-only all-vs-all on their db blocks give bit-for-bit the
    single-process nw_score_all_vs_all, and a sample equals the oracle."""
    import sequencealigning_amd as saln
    from nw_check import rand_seq
    from oracle import refcpu
    rng = np.random.default_rng(21)
    queries = [rand_seq(rng, int(n)) for n in rng.integers(100, 161, 40)] + [b"", b"ACGTN" * 60]
    dbs = [rand_seq(rng, int(n)) for n in rng.integers(100, 161, 57)] + [b"", b"A" * 700]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_avsa_gpu_worker, args=(r, 2, port, queries, dbs, q))
             for r in range(2)]
    for p in procs:
        p.start()
    scores, status = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want_s, want_st = saln.nw_score_all_vs_all(queries, dbs)
    assert np.array_equal(scores, want_s) and np.array_equal(status, want_st)
    for _ in range(30):
        di, qi = int(rng.integers(len(dbs))), int(rng.integers(len(queries)))
        o = refcpu.nw(queries[qi], dbs[di], literal_dfs=False)
        assert scores[di, qi] == o.score and (status[di, qi] == 2) == o.panics


def test_sharded_all_vs_all_without_process_group():
    """One process, no process group (bench.py at N = 1): a single block, the
    gather is a no-op, results and lookups in the reference order."""
    from oracle import refcpu
    from sequencealigning_amd.dist import ShardedAllVsAll
    from sequencealigning_amd.nw import pack_csr
    queries, dbs = [b"ACGT", b"AAC", b""], [b"AC", b"", b"GGTA", b"T"]
    q, qo = pack_csr(queries)
    d, do = pack_csr(dbs)
    s = ShardedAllVsAll(q, qo, d, do, engine=_OracleAvsaEngine)
    s.execute()
    sc, st = s.result()
    for di, dd in enumerate(dbs):
        for qi, qq in enumerate(queries):
            o = refcpu.nw(qq, dd, literal_dfs=False)
            assert sc[di, qi] == o.score and (st[di, qi] == 2) == o.panics
    ls, lst = s.lookup([3, 0, 2], [2, 1, 0])
    assert ls.tolist() == [sc[3, 2], sc[0, 1], sc[2, 0]]


def _nccl_worker(port, queries, dbs, out):
    import torch
    import torch.distributed as dist

    from sequencealigning_amd.dist import nw_align_sharded, nw_score_all_vs_all_sharded
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    sc, st = nw_score_all_vs_all_sharded(queries, dbs, device=0)
    res, cig = nw_align_sharded(queries, dbs, device=0)
    out.put((sc, st, res["score"].copy(), res["status"].copy(), cig))
    dist.destroy_process_group()


@pytest.mark.gpu
def test_rccl_backend_single_rank():
    """The nccl (= RCCL on ROCm) backend path of the multi-GPU drivers, one
    rank on the box's GPU: ShardedAllVsAll's device-buffer gather and status
    all-reduce, and nw_align_sharded's gather_records (all_gather of the
    sizes, gather of the records) all run through RCCL, and the results equal
    the single-process engine's."""
    import sequencealigning_amd as saln
    from nw_check import rand_seq
    rng = np.random.default_rng(22)
    queries = [rand_seq(rng, int(n)) for n in rng.integers(100, 161, 23)] + [b"ACGT" * 300]
    dbs = [rand_seq(rng, int(n)) for n in rng.integers(100, 161, 31)] + [b""]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), queries, dbs, q))
    p.start()
    sc, st, rs, rt, cig = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    want_s, want_st = saln.nw_score_all_vs_all(queries, dbs)
    assert np.array_equal(sc, want_s) and np.array_equal(st, want_st)
    res, want_cig = saln.nw_align_batch(queries, dbs)
    assert np.array_equal(rs, res["score"]) and np.array_equal(rt, res["status"])
    assert cig == want_cig
