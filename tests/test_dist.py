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
