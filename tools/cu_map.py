"""Which CUs a hipExtStreamCreateWithCUMask bit selects on this MI355X
(VERDICT r3 #2), from probe launches (saln_device_cu_probe: each wave's
HW_ID / XCC_ID) on masked streams.

Round 4's first map (profiles/r04_cu_map.json) found that the mask applies per
XCD, bit c selecting a CU of XCD c mod 8, and that an XCD with no bit set runs
UNMASKED (a one-bit mask ran on 225 CUs).  So each bit c is probed with the
other seven bits of its octet set (one CU on every other XCD): the waves on
XCD c mod 8 then sit on bit c's CU alone.  Contiguous ranges are summarised
by the XCDs / SEs they touch; "[0,1) raw" records the leak.  Tools only.

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
    nw = (ncu + 31) // 32

    def mask_stream(bitset):
        words = [0] * nw
        for b in bitset:
            words[b // 32] |= 1 << (b % 32)
        h = C.c_void_p()
        _lib.check(L.saln_stream_create_cu_mask(ctx, (C.c_uint32 * nw)(*words), nw, C.byref(h)),
                   "cu_mask")
        return h

    bits = []
    for c in range(ncu):
        o = c - c % 8
        h = mask_stream(range(o, min(o + 8, ncu)))
        w = probe(L, ctx, h, 256)  # 32 waves per XCD
        L.saln_stream_destroy(ctx, h)
        mine = {(x["xcd"], x["se"], x["sh"], x["cu"]) for x in w if x["xcd"] == c % 8}
        bits.append({"bit": c, "places": sorted(mine)})
    h = mask_stream([0])
    w = probe(L, ctx, h, 2048)
    L.saln_stream_destroy(ctx, h)
    raw1 = {(x["xcd"], x["se"], x["sh"], x["cu"]) for x in w}
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

    ranges = {"[0,1) raw (one bit: its XCD masked, the others unmasked)":
              {"cus": len(raw1), "per_xcd": [sum(1 for p in raw1 if p[0] == x) for x in range(8)]}}
    ranges.update({f"[0,{k})": measured(0, k) for k in (8, 16, 32, 48, 64, 128)})
    ranges.update({f"[{ncu - k},{ncu})": measured(ncu - k, ncu) for k in (16, 32, 64)})
    ranges["[0,256) unmasked probe"] = {"cus": cus_whole}
    places = [tuple(b["places"][0]) for b in bits if len(b["places"]) == 1]
    doc = {"cu_count": ncu, "xcds_unmasked": xcds_whole, "bits": bits, "ranges": ranges,
           "single_place_bits": sum(len(b["places"]) == 1 for b in bits),
           "distinct_places": len(set(places)),
           "bit_xcd_is_bit_mod_8": all(b["places"] and b["places"][0][0] == b["bit"] % 8
                                       for b in bits)}
    print(json.dumps({"cu_count": ncu, "xcds_unmasked": xcds_whole, "ranges": ranges,
                      "places_per_bit": sorted({len(b["places"]) for b in bits}),
                      "distinct_places": doc["distinct_places"],
                      "bit_xcd_is_bit_mod_8": doc["bit_xcd_is_bit_mod_8"],
                      "first_bits": [(b["bit"], b["places"]) for b in bits[:4]]}))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(doc, f, indent=1)


if __name__ == "__main__":
    main()
