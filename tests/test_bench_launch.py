"""CPU: `bench.py --gpus N` starts its own N ranks when no launcher did
(torch.distributed.run on 127.0.0.1, as a child process), and refuses a
WORLD_SIZE that disagrees with --gpus.  gloo, no GPU work (--selftest-launch)."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(kw)
    return env


def test_bench_starts_two_ranks():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--selftest-launch", "--backend", "gloo"], capture_output=True, text=True,
                       env=_env(), timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = [l for l in r.stdout.splitlines() if l.startswith("{")][-1]
    doc = json.loads(line)
    assert doc["launch_selftest"] and doc["n_gpus"] == 2 and doc["ranks"] == [0, 1]
    # the per-rank diagnosis the N > 1 lines carry (bench.rank_diag)
    diag = doc["rank_diag"]
    assert [d["rank"] for d in diag] == [0, 1]
    for d in diag:
        assert set(d) == {"rank", "compute_ms", "gather_ms", "gather_bytes"}
        assert d["compute_ms"] > 0 and d["gather_ms"] > 0
    assert diag[0]["gather_bytes"] == 2 * 4096 * 4 and diag[1]["gather_bytes"] == 4096 * 4


def test_bench_refuses_world_mismatch():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2",
                        "--selftest-launch"], capture_output=True, text=True,
                       env=_env(WORLD_SIZE="3", RANK="0", LOCAL_RANK="0"), timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE=3" in r.stderr


def test_bench_refuses_instrumented_library():
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--legs", "none"],
                       capture_output=True, text=True, env=_env(SALN_LIB="/tmp/x.so"), timeout=120)
    assert r.returncode != 0 and "SALN_LIB" in r.stderr


def test_bench_refuses_leftover_experiment_variables():
    """Any SALN_* variable outside bench.py's allow-list (empty: the engine
    reads none; its tuning goes through saln_option_set) stops the bench
    before it touches the GPU, naming the variable."""
    for var in ("SALN_PK_STEADY", "SALN_ROWS_K", "SALN_ANYTHING"):
        r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--legs", "none"],
                           capture_output=True, text=True, env=_env(**{var: "0"}), timeout=120)
        assert r.returncode != 0 and var in r.stderr, (var, r.stderr[-500:])
    sys.path.insert(0, ROOT)
    import bench
    assert bench.refused_env({"SALN_X": "1", "PATH": "/bin", "XSALN_Y": "2"}) == ["SALN_X"]
    assert bench.refused_env({k: "1" for k in bench.ALLOWED_ENV}) == []


def _c4_sharded_worker(rank, world, port, q, d, out):
    sys.path.insert(0, ROOT)
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import torch
    import torch.distributed as dist

    import bench
    from test_span import _CpuSpanEngine
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r = bench.leg_c4_sharded(world, rank, 0, dist, torch, reps=2, band_rows=64,
                             engine=_CpuSpanEngine, q=q, d=d)
    if rank == 0:
        out.put(r)
    dist.barrier()
    dist.destroy_process_group()


def test_c4_sharded_leg_shape_gloo():
    """at N > 1 bench.py adds the c4_sharded leg (one long pair
    as one column span per rank, span.ShardedLongPair).  Its line on gloo with
    CPU span engines at world 2: per-rank fill / walk / wall / band-exchange
    times, the spans' columns covering the query, and the assembled result
    equal to the oracle's."""
    import multiprocessing as mp
    import socket

    import numpy as np
    sys.path.insert(0, ROOT)
    from oracle import refcpu
    rng = np.random.default_rng(606)
    q = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), 600))
    d = bytearray(q[:520])
    for k in range(0, len(d), 13):
        d[k] = ord("ACGT"[(d[k] + 1) % 4])
    d = bytes(d)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ctx = mp.get_context("spawn")
    out = ctx.Queue()
    procs = [ctx.Process(target=_c4_sharded_worker, args=(r, 2, port, q, d, out)) for r in range(2)]
    for p in procs:
        p.start()
    r = out.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    assert r["n_ranks"] == 2 and r["unit"] == "GCUPS" and r["value"] > 0
    assert [x["rank"] for x in r["per_rank"]] == [0, 1]
    assert sum(x["cols"] for x in r["per_rank"]) == len(q)
    for x in r["per_rank"]:
        assert set(x) == {"rank", "cols", "fill_ms", "walk_ms", "wall_ms", "band_exchange_ms"}
        assert x["fill_ms"] > 0 and x["walk_ms"] > 0 and x["band_exchange_ms"] >= 0
    o = refcpu.nw(q, d, literal_dfs=False)
    assert r["result"]["score"] == o.score and (r["result"]["status"] == 2) == o.panics


def test_gpus1_legs_exclude_c4_sharded():
    """--gpus 1 output is unchanged by the N > 1 leg: it is not an N = 1 leg."""
    sys.path.insert(0, ROOT)
    import bench
    assert "c4_sharded" not in bench.ALL_LEGS
