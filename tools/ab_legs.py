"""A/B timing of bench.py legs for the library SALN_LIB names (an experiment
build) or the in-tree one (tools only; bench.py itself refuses SALN_LIB):
the leg's own workload and timing, without its CPU baseline.

    SALN_LIB=... python tools/ab_legs.py --legs c3,c3_affine [--tag name]
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
    a = ap.parse_args()
    import torch
    import sequencealigning_amd as saln
    from sequencealigning_amd import _lib
    import bench
    for leg in a.legs.split(","):
        r = getattr(bench, "leg_" + leg)(torch, saln, cpu=False)
        print(json.dumps({"tag": a.tag, "lib": os.path.basename(_lib.LIB_PATH), "leg": leg,
                          "value": r.get("value"), "unit": r.get("unit"),
                          "ms": r.get("ms"), "seconds": r.get("seconds"),
                          "verified": r.get("verified")}), flush=True)


if __name__ == "__main__":
    main()
