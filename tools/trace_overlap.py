"""Overlap of the C2 pipeline's kernels in a rocprofv3 kernel trace
(tools/cu_pipeline.py or bench.py under rocprofv3 --kernel-trace
--output-format csv): for each walk (nw_traceback_lds_kernel) the fraction
of its duration during which a fill (nw_fill_pk_kernel / _tab_kernel) ran,
and the fills split into those that overlapped a walk (co-run: the bench's
pipelined kernel_avg_ms) and those that ran alone (kernel_avg_ms_alone:
the bench's sequential executes after its timed region).  Tools only.

    python tools/trace_overlap.py <dir with *kernel_trace.csv> [--out file.json]
"""
import csv
import glob
import json
import os
import sys


def main():
    d = sys.argv[1]
    out = sys.argv[sys.argv.index("--out") + 1] if "--out" in sys.argv else None
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[-1]
    rows = list(csv.DictReader(open(f)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows]
    fills = sorted((s, e) for s, e, n in ks if "nw_fill_pk_kernel" in n or "nw_fill_pk_tab_kernel" in n)
    walks = sorted((s, e) for s, e, n in ks if "nw_traceback_lds_kernel" in n)
    fr = []
    for s, e in walks:
        ov = sum(max(0, min(e, fe) - max(s, fs)) for fs, fe in fills)
        fr.append(ov / max(1, e - s))
    span = (max(e for _, e, _ in ks) - min(s for s, _, _ in ks)) / 1e6
    corun, alone = [], []
    for s, e in fills:
        ov = any(min(e, we) > max(s, ws) for ws, we in walks)
        (corun if ov else alone).append((e - s) / 1e6)
    avg = lambda x: round(sum(x) / len(x), 4) if x else None  # noqa: E731
    # idle time of the fill stream between consecutive pipelined fills (one
    # fill's end to the next one's start, both beside a walk): the hand-off
    # packets between steps (fallback launch, event records and waits)
    co = [(s, e) for s, e in fills if any(min(e, we) > max(s, ws) for ws, we in walks)]
    gaps = sorted((b[0] - a[1]) / 1e3 for a, b in zip(co, co[1:]) if 0 <= b[0] - a[1] < 200e3)
    med = lambda x: round(x[len(x) // 2], 2) if x else None  # noqa: E731
    doc = {"trace": os.path.relpath(f), "walks": len(walks), "fills": len(fills),
           "walk_ms_avg": round(sum(e - s for s, e in walks) / max(1, len(walks)) / 1e6, 4),
           "fill_ms_avg": round(sum(e - s for s, e in fills) / max(1, len(fills)) / 1e6, 4),
           "walk_overlap_frac_avg": round(sum(fr) / max(1, len(fr)), 3),
           "walk_overlap_frac_min": round(min(fr), 3) if fr else None,
           "fill_corun_n": len(corun), "fill_corun_ms_avg": avg(corun),
           "fill_alone_n": len(alone), "fill_alone_ms_avg": avg(alone),
           "fill_gap_us_median": med(gaps), "fill_gap_us_min": round(gaps[0], 2) if gaps else None,
           "fill_gap_n": len(gaps), "trace_span_ms": round(span, 3)}
    print(json.dumps(doc))
    if out:
        json.dump(doc, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
