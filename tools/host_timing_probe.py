"""Stage times of saln_nw_align_batch on configs[1] (host.timing; tools only)."""
import sys, time
sys.path.insert(0, '.')
import numpy as np
import sequencealigning_amd as saln
from sequencealigning_amd import _lib, synth
n = 100_000
qs, qo, ds, do = synth.iid_pairs(n, 150, 150, seed=0x5EED0002)
q = [qs[int(qo[k]):int(qo[k+1])].tobytes() for k in range(n)]
d = [ds[int(do[k]):int(do[k+1])].tobytes() for k in range(n)]
pairs = np.stack([np.arange(n), np.arange(n)], 1)
for k in range(4):
    if k == 3:
        _lib.set_option("host.timing", 1)
    t0 = time.perf_counter()
    saln.nw_align_batch(q, d, pairs=pairs)
    print("wall ms", round((time.perf_counter() - t0) * 1e3, 2), flush=True)
