"""A/B timing harness for the configs[1] step (tools only, never the bench):
the same plan / execute / hipEvent timing as bench.py's headline loop, for
the library SALN_LIB names (an experiment build) or the in-tree one.

    SALN_LIB=... python tools/ab_c2.py [--steps 40] [--warmup 5] [--tag name]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=40)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--pairs", type=int, default=100_000)
    ap.add_argument("--len", type=int, default=150, help="query and db length (150: configs[1])")
    ap.add_argument("--tag", default="")
    ap.add_argument("--pipeline", action="store_true",
                    help="the bench's default loop: step k's walk beside step k+1's fill")
    ap.add_argument("--no-timing", action="store_true",
                    help="no per-execute hipEvents (wall time only)")
    ap.add_argument("--full", action="store_true",
                    help="full parent sets (saln_nw_plan_create_full, the c2_full leg's plan)")
    ap.add_argument("--opt", action="append", default=[],
                    help="engine option name=value (saln_option_set), repeatable")
    a = ap.parse_args()
    import torch
    import sequencealigning_amd as saln
    from sequencealigning_amd import _lib, synth
    for kv in a.opt:
        k, v = kv.split("=")
        _lib.set_option(k, int(v))
    n, L = a.pairs, a.len
    qs, qo, ds, do = synth.iid_pairs(n, L, L, seed=0x5EED0002)
    plan = saln.NwPlan(qo, do, pairs=np.stack([np.arange(n)] * 2, 1), full_codes=a.full)
    dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
    nb = 2 if a.pipeline else 1
    plan.set_async(a.pipeline)
    res = [torch.zeros(n * 4, dtype=torch.int32, device="cuda") for _ in range(nb)]
    cig = [torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
           for _ in range(nb)]

    def run(k):
        for i in range(k):
            plan.execute(dq, dd, res[i % nb], cig[i % nb])
        if a.pipeline:
            plan.sync()
        torch.cuda.synchronize()
    run(a.warmup)
    plan.set_timing(not a.no_timing)
    t0 = time.perf_counter()
    run(a.steps)
    dt = (time.perf_counter() - t0) / a.steps
    plan.check()
    f, fn = plan.kernel_time("nw_fill") if not a.no_timing else (0.0, 1)
    tb, tn = plan.kernel_time("nw_traceback") if not a.no_timing else (0.0, 1)
    print(json.dumps({"tag": a.tag, "lib": os.path.basename(_lib.LIB_PATH), "opts": a.opt,
                      "timing": not a.no_timing,
                      "pipeline": a.pipeline, "full": a.full,
                      "gcups": round(plan.cells / dt / 1e9, 1), "ms_per_step": round(dt * 1e3, 4),
                      "fill_ms": round(f / fn, 4), "traceback_ms": round(tb / tn, 4)}))


if __name__ == "__main__":
    main()
