"""configs[3]'s pair as n column spans on one GPU (span.py SpanChain, the
bench's c4_spans setup): `--reps` pipelined fills only, for a rocprofv3
--kernel-trace of the chain; `--report DIR` instead prints, for the last
chain in DIR's kernel trace, each fill and relay kernel's start / end (ms from
the chain's first start), queue and duration.  Tools only (the
4-span anomaly).

    rocprofv3 --kernel-trace -d OUT -o run --output-format csv -- python3 tools/span_trace.py --spans 4
    python3 tools/span_trace.py --report OUT --spans 4
"""
import argparse
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def report(d, n):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[-1]
    rows = list(csv.DictReader(open(f)))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"],
                 r["Queue_Id"], r.get("Grid_Size_X")) for r in rows
                if "nw_fill_rows_kernel" in r["Kernel_Name"] or "relay" in r["Kernel_Name"])
    fills = [k for k in ks if "nw_fill_rows" in k[2]]
    last = fills[-n:]  # the last chain's n fills
    t0 = min(k[0] for k in last)
    sel = [k for k in ks if k[0] >= t0 - 1_000_000]
    out = []
    for s, e, name, q, grid in sel:
        out.append({"kernel": "fill" if "fill" in name else "relay", "queue": q, "grid": grid,
                    "start_ms": round((s - t0) / 1e6, 3), "end_ms": round((e - t0) / 1e6, 3),
                    "ms": round((e - s) / 1e6, 3)})
    print(json.dumps({"trace": os.path.relpath(f), "spans": n, "kernels": out}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spans", type=int, default=4)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--band-rows", type=int, default=1024)
    ap.add_argument("--report", default=None)
    ap.add_argument("--solo", action="store_true",
                    help="fill span 0 alone on its CU-masked stream (the other spans idle)")
    a = ap.parse_args()
    if a.report:
        report(a.report, a.spans)
        return
    import torch
    from sequencealigning_amd import synth
    from sequencealigning_amd.span import SpanChain
    q = synth.random_bases(0x5EED0003, 100_000).tobytes()
    d = synth.mutate(q, 0.05, seed=100_000)
    ch = SpanChain(q, d, a.spans, band_rows=a.band_rows)
    ms = []
    for _ in range(a.reps):
        torch.cuda.synchronize()
        if a.solo:
            main = torch.cuda.current_stream()
            s0 = ch.spans[0]
            s0.reset(main)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main)
            st = torch.cuda.ExternalStream(ch.cu_streams[0].value)
            st.wait_event(e0)
            s0.fill(ch.q, ch.d, ch.cu_streams[0].value)
            e1.record(st)
            torch.cuda.synchronize()
            s0.check()
            ms.append(e0.elapsed_time(e1))
        else:
            ch.fill(pipelined=True)
            torch.cuda.synchronize()
    if not a.solo:
        ch.check()
    ch.close()
    print(json.dumps({"spans": a.spans, "reps": a.reps, "solo_span0_ms": ms, "ok": True}))


if __name__ == "__main__":
    main()
