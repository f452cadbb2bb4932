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

cases = [(int(a), int(b)) for a, b in (x.split(":") for x in
                                       (sys.argv[1] if len(sys.argv) > 1 else "1:4096,8:4096").split(","))]
for n, b in cases:
    r = bench.leg_c4_spans(torch, saln, n_spans=n, reps=3, band_rows=b)
    print(os.environ.get("GPU_MAX_HW_QUEUES"), n, b, json.dumps(r), flush=True)
