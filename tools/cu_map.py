"""Which CUs a hipExtStreamCreateWithCUMask bit selects on this MI355X
(VERDICT r3 #2): for every mask bit c, a stream on CU c alone runs a probe
launch (saln_device_cu_probe: each wave's HW_ID / XCC_ID), giving the bit ->
(XCD, SE, SH, CU) order; then contiguous ranges [0, n) and the strided
ranges are summarised by the XCDs / SEs they touch.  Tools only.

    python tools/cu_map.py [--out profiles/r04_cu_map.json]
"""
import argparse
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def decode(hw, xcc):
    return {"xcd": xcc & 0xF, "se": (hw >> 13) & 7, "sh": (hw >> 12) & 1, "cu": (hw >> 8) & 0xF,
            "simd": (hw >> 4) & 3}


def probe(L, ctx, stream, n):
    hw = (C.c_uint32 * n)()
    xc = (C.c_uint32 * n)()
    rc = L.saln_device_cu_probe(ctx, stream, n, hw, xc)
    if rc != 0:
        raise RuntimeError(f"probe rc {rc}")
    return [decode(hw[k], xc[k]) for k in range(n)]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    import torch  # noqa: F401  (HIP runtime shared with torch)
    from sequencealigning_amd import _lib
    L, ctx = _lib.lib(), _lib.context(0)
    n = C.c_uint32()
    _lib.check(L.saln_device_cu_count(ctx, C.byref(n)), "cu_count")
    ncu = n.value
    bits = []
    for c in range(ncu):
        h = C.c_void_p()
        _lib.check(L.saln_stream_create_cu_range(ctx, c, c + 1, C.byref(h)), "cu_range")
        w = probe(L, ctx, h, 64)  # 64 waves: more than one per XCD if the bit allows it
        L.saln_stream_destroy(ctx, h)
        places = {(x["xcd"], x["se"], x["sh"], x["cu"]) for x in w}
        bits.append({"bit": c, "places": sorted(places)})
    whole = probe(L, ctx, None, 4096)
    xcds_whole = sorted({x["xcd"] for x in whole})
    cus_whole = len({(x["xcd"], x["se"], x["sh"], x["cu"]) for x in whole})

    def measured(lo, hi, n=2048):
        h = C.c_void_p()
        _lib.check(L.saln_stream_create_cu_range(ctx, lo, hi, C.byref(h)), "cu_range")
        w = probe(L, ctx, h, n)
        L.saln_stream_destroy(ctx, h)
        pl = {(x["xcd"], x["se"], x["sh"], x["cu"]) for x in w}
        return {"cus": len(pl), "xcds": len({p[0] for p in pl}),
                "xcd_se": len({(p[0], p[1]) for p in pl}),
                "per_xcd": [sum(1 for p in pl if p[0] == x) for x in range(8)]}

    ranges = {f"[0,{k})": measured(0, k) for k in (1, 8, 16, 32, 48, 64, 128)}
    ranges.update({f"[{ncu - k},{ncu})": measured(ncu - k, ncu) for k in (16, 32, 64)})
    ranges["[0,256) unmasked probe"] = {"cus": cus_whole}
    doc = {"cu_count": ncu, "xcds_unmasked": xcds_whole, "bits": bits, "ranges": ranges,
           "single_place_bits": sum(len(b["places"]) == 1 for b in bits)}
    print(json.dumps({"cu_count": ncu, "xcds_unmasked": xcds_whole, "ranges": ranges,
                      "places_per_bit": sorted({len(b["places"]) for b in bits}),
                      "first_bits": [(b["bit"], b["places"]) for b in bits[:4]]}))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
