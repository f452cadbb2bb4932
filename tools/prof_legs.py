"""Profiling driver for bench.py's legs (c2_full, c1, c3, c3_affine, c4, c5): each
leg's GPU workload exactly as the bench runs it, without its CPU baseline and
checks; used under rocprofv3 (--kernel-trace --stats, and the --pmc passes of
tools/pmc.sh).  Writes {leg: executes} (runs of the leg's workload) to
$PMC_EXECUTES (default gpurun_out/pmc/executes.json) so tools/pmc_traffic.py
can turn the counters' per-run sums into per-execute figures.

    python tools/prof_legs.py [--legs c2_full,c1,c3,c3_affine,c4,c4_spans,c5] [--opt name=value ...]

--opt sets engine options (saln_option_set) for the whole run, e.g.
nw.rows_xcd=0 for the C4 row fill's traffic without XCD-local stripes.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def c4_spans_serial(torch, n_spans=8, reps=3):
    """bench.py's c4_spans fills for the PMC passes: rocprofv3 --pmc runs one
    kernel at a time, so the chain's concurrent span fills and relays (span
    r + 1 polls rows that span r publishes) cannot run under it.  Here the
    spans fill one after another, each on its own CU-masked stream as in the
    chain (the same kernel instantiation, one stripe per SIMD of its CUs),
    its inbox copied from the previous span's outbox: the same mask and
    boundary bytes per span launch."""
    from sequencealigning_amd import synth
    from sequencealigning_amd.span import SpanChain
    q = synth.random_bases(0x5EED0003, 100_000).tobytes()
    d = synth.mutate(q, 0.05, seed=100_000)
    ch = SpanChain(q, d, n_spans, band_rows=1024, edge_masks="shared")
    main = torch.cuda.current_stream()
    for _ in range(1 + reps):
        for s in ch.spans:
            s.reset(main)
        for r, s in enumerate(ch.spans):
            if r:
                s.inbox.copy_(ch.spans[r - 1].outbox)
            torch.cuda.synchronize()
            s.fill(ch.q, ch.d, ch.cu_streams[r].value)
            torch.cuda.synchronize()
            s.check()
    ch.close()
    return {"executes": 1 + reps, "spans": n_spans}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--legs", default="c2_full,c1,c3,c3_affine,c4,c5")
    ap.add_argument("--opt", action="append", default=[],
                    help="engine option name=value (saln_option_set), repeatable")
    a = ap.parse_args()
    import torch
    import sequencealigning_amd as saln
    import bench
    from sequencealigning_amd import _lib
    for kv in a.opt:
        k, v = kv.split("=")
        _lib.set_option(k, int(v))
    ex = {}
    for leg in a.legs.split(","):
        if leg == "c5":
            r = bench.leg_c5(1, 0, 0, None, torch, cpu=False)
        elif leg == "c2_full":
            r = bench.leg_c2_full(torch, saln)
        elif leg == "c1":
            r = bench.leg_c1(torch, saln, cpu=False)
        elif leg == "c3":
            r = bench.leg_c3(torch, saln, cpu=False)
        elif leg == "c3_affine":
            r = bench.leg_c3_affine(torch, saln, cpu=False)
        elif leg == "c4":
            r = bench.leg_c4(torch, saln, cpu=False)
        elif leg == "c4_spans":
            r = c4_spans_serial(torch)
        else:
            raise SystemExit(f"unknown leg {leg}")
        ex[leg] = r["executes"]
        print(leg, json.dumps(r)[:400], flush=True)
    path = os.environ.get("PMC_EXECUTES", os.path.join(ROOT, "gpurun_out", "pmc", "executes.json"))
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as fh:
        json.dump(ex, fh)


if __name__ == "__main__":
    main()
