"""A/B timing of bench.py legs for the library SALN_LIB names (an experiment
build) or the in-tree one (tools only; bench.py itself refuses SALN_LIB):
the leg's own workload and timing, without its CPU baseline.

    SALN_LIB=... python tools/ab_legs.py --legs c3,c3_affine [--tag name] [--opt name=value]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--legs", default="c3")
    ap.add_argument("--tag", default="")
    ap.add_argument("--opt", action="append", default=[],
                    help="engine option name=value (saln_option_set), repeatable")
    a = ap.parse_args()
    import torch
    import sequencealigning_amd as saln
    from sequencealigning_amd import _lib
    import bench
    for kv in a.opt:
        k, v = kv.split("=")
        _lib.set_option(k, int(v))
    for leg in a.legs.split(","):
        fn = getattr(bench, "leg_" + leg)
        r = fn(torch, saln) if leg == "c4_spans" else fn(torch, saln, cpu=False)
        print(json.dumps({"tag": a.tag, "lib": os.path.basename(_lib.LIB_PATH), "leg": leg,
                          "value": r.get("value"), "unit": r.get("unit"),
                          "ms": r.get("ms"), "seconds": r.get("seconds"),
                          "fill_ms": r.get("fill_ms"), "walk_ms": r.get("walk_ms"),
                          "opts": a.opt,
                          "verified": r.get("verified")}), flush=True)


if __name__ == "__main__":
    main()
