"""C4 pair as column spans on one GPU (bench.leg_c4_spans) over span counts
and band sizes; run under different GPU_MAX_HW_QUEUES to see the queue
sharing of the spans' streams."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import bench  # noqa: E402
import sequencealigning_amd as saln  # noqa: E402

# cases "spans:band_rows[:edge_masks[:width]]" (edge_masks shared | unique, span.py
# SpanChain; width: CUs per span's mask, span r on bits [r*width, (r+1)*width),
# default 256 / spans)
for o in [x for x in sys.argv[2:] if "=" in x]:  # engine options name=value (A/Bs)
    k, v = o.split("=")
    saln.set_option(k, int(v))
cases = [x.split(":") for x in (sys.argv[1] if len(sys.argv) > 1 else "1:4096,8:4096").split(",")]
for c in cases:
    n, b, em = int(c[0]), int(c[1]), (c[2] if len(c) > 2 else "shared")
    w = int(c[3]) if len(c) > 3 else 0
    rng = [(r * w, (r + 1) * w) for r in range(n)] if w else None
    r = bench.leg_c4_spans(torch, saln, n_spans=n, reps=3, band_rows=b, edge_masks=em,
                           cu_ranges=rng)
    print(os.environ.get("GPU_MAX_HW_QUEUES"), n, b, em, w or None, json.dumps(r), flush=True)
