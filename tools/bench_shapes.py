"""NW-affine throughput for arbitrary pair shapes through a device-resident
plan (which fill variant runs depends on the shape: packed i16 inside the
packed region, i32 lanes up to 512 query columns, column stripes above).

    python tools/bench_shapes.py --shape 150x1000 --pairs 20000 [--shape ...]
"""
import argparse
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(saln, synth, torch, lq, ld, n, reps, score_only):
    qs, qo, ds, do = synth.iid_pairs(n, lq, ld, seed=0x5EED0009)
    plan = saln.NwPlan(qo, do, pairs=np.stack([np.arange(n), np.arange(n)], 1))
    plan.set_score_only(score_only)
    dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
    res = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
    cig = torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
    plan.execute(dq, dd, res, cig)
    torch.cuda.synchronize()
    plan.set_timing(True)
    for _ in range(reps):
        plan.execute(dq, dd, res, cig)
    torch.cuda.synchronize()
    f_ms, f_n = plan.kernel_time("nw_fill")
    t_ms, t_n = plan.kernel_time("nw_traceback")
    e_ms, e_n = plan.kernel_time("nw_execute")
    cells = float(lq) * ld * n
    out = {"shape": f"{lq}x{ld}", "pairs": n, "score_only": score_only,
           "fill_ms": round(f_ms / max(1, f_n), 3), "traceback_ms": round(t_ms / max(1, t_n), 3),
           "execute_ms": round(e_ms / max(1, e_n), 3),
           "gcups": round(cells / (e_ms / max(1, e_n) / 1e3) / 1e9, 1)}
    plan.close()
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--shape", action="append", default=[])
    ap.add_argument("--pairs", type=int, default=20000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--score-only", action="store_true")
    a = ap.parse_args()
    import torch
    import sequencealigning_amd as saln
    from sequencealigning_amd import synth
    for sh in a.shape or ["150x1000"]:
        lq, ld = (int(x) for x in sh.split("x"))
        print(json.dumps(run(saln, synth, torch, lq, ld, a.pairs, a.reps, a.score_only)), flush=True)


if __name__ == "__main__":
    main()
