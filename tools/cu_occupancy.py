"""Where a CU-masked launch of one-wave workgroups puts its waves (VERDICT r3
#2, the span-chain anomaly): for mask ranges [0, W) and grids of G waves (the
span fills' shapes), the number of waves per SIMD and per CU from the probe's
HW_ID (saln_device_cu_probe).  Tools only.

    python tools/cu_occupancy.py [W:G ...]   (default 32:98 64:196 128:391 256:782)
"""
import collections
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    import torch  # noqa: F401
    from sequencealigning_amd import _lib
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    from cu_map import decode
    L, ctx = _lib.lib(), _lib.context(0)
    cases = [tuple(int(x) for x in c.split(":")) for c in
             (sys.argv[1:] or ["32:98", "64:196", "128:391", "256:782"])]
    for w, g in cases:
        h = C.c_void_p()
        _lib.check(L.saln_stream_create_cu_range(ctx, 0, w, C.byref(h)), "cu_range")
        hw = (C.c_uint32 * g)()
        xc = (C.c_uint32 * g)()
        _lib.check(L.saln_device_cu_probe(ctx, h, g, hw, xc), "probe")
        L.saln_stream_destroy(ctx, h)
        pl = [decode(hw[k], xc[k]) for k in range(g)]
        simd = collections.Counter((p["xcd"], p["se"], p["sh"], p["cu"], p["simd"]) for p in pl)
        cu = collections.Counter((p["xcd"], p["se"], p["sh"], p["cu"]) for p in pl)
        print(json.dumps({"mask_cus": w, "waves": g, "cus_used": len(cu), "simds_used": len(simd),
                          "waves_per_simd": dict(sorted(collections.Counter(simd.values()).items())),
                          "waves_per_cu": dict(sorted(collections.Counter(cu.values()).items()))}),
              flush=True)


if __name__ == "__main__":
    main()
