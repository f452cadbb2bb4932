"""Debug: row fill vs oracle on a few shapes, per SALN_ROWS_K (set by caller)."""
import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))
import numpy as np
import sequencealigning_amd as saln
from oracle import refcpu
from nw_check import rand_seq
os.environ["SALN_STRIPE_PK"] = "0"
rng = np.random.default_rng(2024)
for lq, ld, n in [(1100, 250, 1), (1100, 252, 1), (600, 17, 1), (1100, 250, 3), (1100, 250, 40), (700, 1000, 5)]:
    qs = [rand_seq(rng, lq) for _ in range(n)]
    ds = [rand_seq(rng, ld) for _ in range(n)]
    res, cig = saln.nw_align_batch(qs, ds, pairs=[(k, k) for k in range(n)])
    bad = []
    for k in range(n):
        o = refcpu.nw(qs[k], ds[k], literal_dfs=False)
        if int(res["score"][k]) != o.score:
            bad.append((k, int(res["score"][k]), o.score))
    print(os.environ.get("SALN_ROWS_K"), lq, ld, n, "bad", len(bad), bad[:3], flush=True)
