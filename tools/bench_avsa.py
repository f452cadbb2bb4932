"""configs[4] (C5) slice: score-only all-vs-all, n_q queries x n_db db records
of 150 bp (G-iid, seed 0x5EED0004), sequences resident in HBM, results
{score, status} per pair in the reference order.  Reports GCUPS, pairs/s and
the time the full 10^4 x 10^5 run would take at that rate.

    python tools/bench_avsa.py [--nq 1000] [--ndb 100000] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--nq", type=int, default=1000)
    ap.add_argument("--ndb", type=int, default=100_000)
    ap.add_argument("--len", type=int, default=150)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--opt", action="append", default=[], help="engine option name=value (A/Bs)")
    ap.add_argument("--check", action="store_true", help="compare every result with nw.avsa_profile=0")
    a = ap.parse_args()
    import torch
    import sequencealigning_amd as saln
    for o in a.opt:
        k, v = o.split("=")
        saln.set_option(k, int(v))
    from sequencealigning_amd import synth
    seed = 0x5EED0004
    L = a.len
    qs = synth.random_bases(seed, a.nq * L)
    ds = synth.random_bases(seed ^ 0xD5D5D5D5, a.ndb * L)
    qo = np.arange(a.nq + 1, dtype=np.uint64) * np.uint64(L)
    do = np.arange(a.ndb + 1, dtype=np.uint64) * np.uint64(L)
    t0 = time.perf_counter()
    av = saln.NwAllVsAll(qo, do)
    setup = time.perf_counter() - t0
    dq = torch.from_numpy(qs).cuda()
    dd = torch.from_numpy(ds).cuda()
    out = torch.empty(a.nq * a.ndb * 2, dtype=torch.int32, device="cuda")
    av.execute(dq, dd, out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        av.execute(dq, dd, out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    pairs = a.nq * a.ndb
    same = None
    if a.check:  # the same plan's results with the profile path off (run with nw.avsa_profile=1)
        ref = torch.empty_like(out)
        with saln.options(**{"nw.avsa_profile": 0}):
            av.execute(dq, dd, ref)
        torch.cuda.synchronize()
        same = bool(torch.equal(out, ref))
    h = out[: 2 * min(pairs, 1 << 20)].cpu().numpy().reshape(-1, 2)
    full_cells = 10_000 * 100_000 * L * L
    gcups = av.cells / dt / 1e9
    print(json.dumps({"workload": f"configs[4] slice: {a.nq} x {a.ndb} score-only all-vs-all, "
                                  f"{L} bp G-iid", "pairs": pairs, "cells": av.cells,
                      "fallback_pairs": av.fallback_pairs, "plan_s": round(setup, 3),
                      "ms": round(dt * 1e3, 3), "gcups": round(gcups, 1), "pairs_per_s": round(pairs / dt, 1),
                      "full_c5_s_at_this_rate_1gpu": round(full_cells / (gcups * 1e9), 1),
                      "panic_frac_sample": round(float((h[:, 1] == 2).mean()), 4),
                      "opts": a.opt, "equal_without_profile": same}))
    av.close()


if __name__ == "__main__":
    main()
