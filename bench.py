#!/usr/bin/env python3
"""Headline benchmark: GCUPS of the NW-affine hot path on MI355X.

Workload (BASELINE.json configs[1]): 100,000 independent 150 x 150 G-iid DNA
pairs per GPU (seed 0x5EED0002 + rank), sequences resident in HBM.  One step
= one pass of the hot path over the batch: NW-affine matrix fill with the
1 B/cell parent mask (nw_fill) + the reference's first-printed traceback per
pair -> score, panic status, CIGAR (nw_traceback); with N > 1 ranks also the
RCCL gather of the 16-byte per-pair result records to rank 0 (db sharded,
SURVEY.md §8(e)).  value = all ranks' cells / max-over-ranks wall time.

    python bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GCUPS (affine-gap NW) at 1/2/4/8 MI355X; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
VALU_PEAK_TOPS = 1024 * 16 * 2.4e9 / 1e12  # 39.3: 256 CUs x 4 SIMDs x 16 lanes x 2.4 GHz
N_PAIRS, LQ, LD = 100_000, 150, 150
SEED = 0x5EED0002


def cpu_threads() -> int:
    """Host threads for the CPU baseline: the box's CPU share (OMP_NUM_THREADS
    is set to it on the GPU pool; os.cpu_count() shows the whole machine)."""
    n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, min(n, 16))


def cpu_baseline(budget_s: float = 12.0) -> dict:
    """Oracle (C port of the reference CPU path: full 3-matrix fill with
    parent sets + the reference's exhaustive DFS traceback) on a bounded
    sample of the same workload: one core for ~budget/3 (the reference's own
    sequential loop, main.rs:61-67), then the same port over pairs on all of
    the box's cores for ~2*budget/3."""
    from oracle import refcpu  # cpu_baseline leg only
    from sequencealigning_amd import synth
    refcpu.build()
    n = 60000
    qs, qo, ds, do = synth.iid_pairs(n, LQ, LD, seed=SEED)
    qb, db = qs.tobytes(), ds.tobytes()
    done = cells = 0
    t0 = time.perf_counter()
    while done < n and time.perf_counter() - t0 < budget_s / 3:
        k = min(64, n - done)
        cells += refcpu.run_pairs(qb[done * LQ:(done + k) * LQ], qo[:k + 1],
                                  db[done * LD:(done + k) * LD], do[:k + 1], k, max_pops=100_000)
        done += k
    dt1 = time.perf_counter() - t0
    rate1 = cells / dt1  # cells/s on one core
    T = cpu_threads()
    # pairs for ~2/3 of the budget at T x the one-core rate (sublinear scaling only shortens it)
    n_mt = int(min(n, max(T * 64, rate1 * T * (2 * budget_s / 3) / (LQ * LD))))
    t0 = time.perf_counter()
    cells_mt = refcpu.run_pairs_mt(qb[:n_mt * LQ], qo[:n_mt + 1], db[:n_mt * LD], do[:n_mt + 1],
                                   n_mt, max_pops=100_000, threads=T)
    dtm = time.perf_counter() - t0
    return {"value": round(cells_mt / dtm / 1e9, 6), "unit": "GCUPS", "cores": T, "kind": "port",
            "value_1core": round(rate1 / 1e9, 6),
            "sample": f"{n_mt} of the 150x150 G-iid pairs (seed {SEED:#x}) on {T} threads in "
                      f"{dtm:.1f} s, {done} pairs on 1 thread in {dt1:.1f} s; oracle/refcpu.c "
                      f"fill + literal DFS (<=1e5 pops/pair)"}


def pmc_traffic(kernel: str, field: str = "hbm_bytes"):
    """A per-launch PMC figure of `kernel` (HBM bytes, or VALU wave-instructions
    with field="valu_wave_insts") from the committed PMC summary
    (profiles/pmc_traffic.json, written by tools/pmc_traffic.py from the
    rocprofv3 --pmc passes of tools/pmc.sh on this workload), or None."""
    try:
        with open(os.path.join(ROOT, "profiles", "pmc_traffic.json")) as fh:
            doc = json.load(fh)
    except (OSError, ValueError):
        return None
    for name, v in doc.get("kernels", {}).items():
        if kernel in name:
            return v.get(field)
    return None


def valu_roof(kernel: str, avg_s: float):
    """SURVEY.md 8(d) asks for the VALU fraction beside the HBM one: the fill's
    VALU wave-instructions per launch (PMC SQ_INSTS_VALU) x 64 lanes over its
    measured duration, against 1,024 SIMDs x 16 lanes x 2.4 GHz (one wave64
    instruction per 4 cycles per SIMD; the 2-cycle ops the kernel favours can
    exceed that rate, so frac may approach or pass 1 when issue-bound)."""
    n = pmc_traffic(kernel, "valu_wave_insts")
    if not n:
        return None
    achieved = n * 64 / avg_s / 1e12
    return {"wave_insts_per_launch": n, "achieved": round(achieved, 2),
            "peak": VALU_PEAK_TOPS, "unit": "T int lane-ops/s", "frac": round(achieved / VALU_PEAK_TOPS, 4)}


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=N_PAIRS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--score-only", action="store_true",
                    help="score + panic status only (no parent codes / traceback; the C5 mode)")
    ap.add_argument("--pipeline", action="store_true",
                    help="overlap step k's traceback with step k+1's fill on a second stream "
                         "(measured slower on MI355X: the walk slows the VALU-bound fill)")
    args = ap.parse_args()

    import torch
    import torch.distributed as dist

    import sequencealigning_amd as saln
    from sequencealigning_amd import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))

    n = args.pairs
    qs, qo, ds, do = synth.iid_pairs(n, LQ, LD, seed=SEED + rank)
    plan = saln.NwPlan(qo, do, pairs=np.stack([np.arange(n), np.arange(n)], 1), device=local)
    dq = torch.from_numpy(qs).to(f"cuda:{local}")
    dd = torch.from_numpy(ds).to(f"cuda:{local}")
    # --pipeline: the traceback of step k runs on the engine's second stream
    # while step k+1 fills; results/cigar/mask are double-buffered and every
    # step's results are complete (and gathered) inside the timed region.
    pipelined = args.pipeline and not args.score_only
    plan.set_score_only(args.score_only)
    plan.set_async(pipelined)
    nbuf = 2 if pipelined else 1
    res = [torch.zeros(n * 4, dtype=torch.int32, device=f"cuda:{local}") for _ in range(nbuf)]
    cig = [torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device=f"cuda:{local}")
           for _ in range(nbuf)]
    gathered = ([torch.empty_like(res[0]) for _ in range(world)] if (world > 1 and rank == 0)
                else None)
    state = {"k": 0}

    def gather(buf):
        if world > 1:
            dist.gather(res[buf], gathered, dst=0)

    def step():
        k = state["k"]
        buf = k % nbuf
        plan.execute(dq, dd, res[buf], cig[buf])
        state["k"] = k + 1
        if pipelined:
            if k > 0 and world > 1:
                plan.sync(keep_latest=True)  # results of step k-1 are complete
                gather((k - 1) % nbuf)
        else:
            gather(buf)

    def drain():
        if pipelined:
            plan.sync()
            if state["k"] > 0:
                gather((state["k"] - 1) % nbuf)
        state["k"] = 0

    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    plan.set_timing(True)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    drain()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    fill_ms, fill_n = plan.kernel_time("nw_fill")
    tb_ms, tb_n = plan.kernel_time("nw_traceback")
    ex_ms, ex_n = plan.kernel_time("nw_execute")
    t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dt = float(t.item())
    cells_rank = plan.cells
    total_cells = cells_rank * world * args.steps
    gcups = total_cells / dt / 1e9
    fill_avg_s = fill_ms / max(1, fill_n) / 1e3
    achieved = cells_rank * 1.0 / fill_avg_s / 1e9  # 1 B/cell parent mask, GB/s
    if rank == 0:
        hr = res[(args.steps - 1) % nbuf].cpu().numpy()
        statuses = np.bincount(hr[1::4] & 0xFF, minlength=3)
        out = {
            "metric": METRIC, "value": round(gcups, 3), "unit": "GCUPS", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "int16x2",
            "data": "synthetic (splitmix64 G-iid ACGT)",
            "config": {"workload": ("configs[1]: independent 150x150 NW-affine pairs per GPU "
                                    "(fill + 1 B/cell parent mask + first-printed traceback/CIGAR)")
                       if not args.score_only else
                       ("score-only 150x150 NW-affine pairs per GPU (the configs[4] per-pair "
                        "mode: score + panic status, no mask)"),
                       "pairs_per_gpu": n, "len_q": LQ, "len_db": LD, "seed": hex(SEED),
                       "parallelism": f"db-sharded x{world}" + (" + RCCL gather" if world > 1
                                                               else "")},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": pmc_traffic("nw_fill_pk_kernel<16, 10,") if not args.score_only else None,
                         "traffic_unit": "bytes/launch (PMC FETCH_SIZE*2 + WRITE_SIZE)",
                         "algorithmic_bytes": cells_rank, "kernel": "nw_fill",
                         "kernel_avg_ms": round(fill_avg_s * 1e3, 4),
                         "traceback_avg_ms": round(tb_ms / max(1, tb_n), 4),
                         "execute_avg_ms": round(ex_ms / max(1, ex_n), 4),
                         "pipelined": pipelined,
                         "valu": valu_roof("nw_fill_pk_kernel<16, 10,", fill_avg_s)
                         if not args.score_only else None},
            "status_counts": {"ok": int(statuses[0]), "ref_panic_boundary": int(statuses[2])},
        }
        if not args.no_cpu_baseline and world == 1:  # the CPU leg: rank 0 at N = 1 only
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out), flush=True)
    plan.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
