"""configs[1] through the host-buffer boundary (saln_nw_align_batch): the
PCIe-inclusive rate a caller with host arrays sees (plan + H2D of the
sequences + fill + traceback + D2H of results and CIGARs), next to the
HBM-resident rate bench.py reports.  Never the bench value.

    python tools/bench_host.py [--pairs 100000] [--reps 3]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=100_000)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--opt", action="append", default=[], help="engine option name=value")
    a = ap.parse_args()
    import sequencealigning_amd as saln
    for o in a.opt:
        k, v = o.split("=")
        saln.set_option(k, int(v))
    from sequencealigning_amd import _lib, synth
    qs, qo, ds, do = synth.iid_pairs(a.pairs, 150, 150, seed=0x5EED0002)
    pq = np.arange(a.pairs, dtype=np.uint32)
    res = np.zeros(a.pairs, dtype=_lib.RESULT_DTYPE)
    coff = np.zeros(a.pairs + 1, np.uint64)
    coff[1:] = np.cumsum(np.full(a.pairs, 300, np.uint64))
    cig = np.zeros(int(coff[-1]), np.uint32)
    vp = lambda x: x.ctypes.data_as(C.c_void_p)  # noqa: E731
    L, ctx = _lib.lib(), _lib.context(0)

    def run():
        _lib.check(L.saln_nw_align_batch(ctx, vp(qs), vp(qo), a.pairs, vp(ds), vp(do), a.pairs,
                                         vp(pq), vp(pq), a.pairs, 0, None, vp(res), vp(cig),
                                         vp(coff)), "saln_nw_align_batch")
    run()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        run()
    dt = (time.perf_counter() - t0) / a.reps
    cells = 150 * 150 * a.pairs
    print(json.dumps({"workload": f"configs[1] via saln_nw_align_batch (host buffers): {a.pairs} "
                                  "150x150 G-iid pairs, score + status + first alignment CIGAR",
                      "ms": round(dt * 1e3, 2), "gcups_pcie_inclusive": round(cells / dt / 1e9, 1),
                      "note": "includes plan creation, H2D, both kernels, D2H; bench.py's value "
                              "is the HBM-resident rate"}))


if __name__ == "__main__":
    main()
