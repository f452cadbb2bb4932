"""Profiling driver: one plan over the bench workload, executed a few times
(used under rocprofv3 --pmc; no timing of its own)."""
import argparse
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100_000)
    ap.add_argument("--len", type=int, default=150)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--opt-sets", default="",
                    help="';'-separated option sets (name=value,...): one plan per set, "
                         "each created under its options (e.g. 'nw.pk_tab=1;nw.pk_tab=2')")
    a = ap.parse_args()
    import torch
    import sequencealigning_amd as saln
    from sequencealigning_amd import _lib, synth
    qs, qo, ds, do = synth.iid_pairs(a.pairs, a.len, a.len, seed=0x5EED0002)
    dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
    res = torch.zeros(a.pairs * 4, dtype=torch.int32, device="cuda")
    for opts in (a.opt_sets.split(";") if a.opt_sets else [""]):
        _lib.lib().saln_options_reset()
        for kv in filter(None, opts.split(",")):
            k, v = kv.split("=")
            _lib.set_option(k, int(v))
        plan = saln.NwPlan(qo, do, pairs=np.stack([np.arange(a.pairs)] * 2, 1))
        cig = torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
        for _ in range(a.reps):
            plan.execute(dq, dd, res, cig)
        torch.cuda.synchronize()
        plan.close()
        print(opts or "defaults", "mask bytes", plan.mask_bytes, "cells", plan.cells)


if __name__ == "__main__":
    main()
