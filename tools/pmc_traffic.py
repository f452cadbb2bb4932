"""HBM traffic (and, when that pass ran, VALU / SALU instruction counts) per
launch from the rocprofv3 --pmc passes of tools/pmc.sh.

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch.  On gfx950 FETCH_SIZE counts
half the bytes of wide streaming reads (MI355X_MICROARCH.md, HBM section), so
reads are doubled; WRITE_SIZE is taken as is (the fill's dwordx3 stores were
checked against the plan's exact mask byte count).  Writes the per-kernel mean
to profiles/pmc_traffic.json, which bench.py reports as roofline.traffic."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


SOURCES = {
    "nw": "tools/pmc.sh (rocprofv3 --pmc, one counter group per pass) on tools/prof_nw.py: "
          "100000 x 150x150 G-iid pairs, seed 0x5EED0002",
    "legs": "tools/pmc.sh (rocprofv3 --pmc, one counter group per pass) on tools/prof_legs.py: "
            "bench.py's legs without their CPU parts; executes = runs of each leg's workload "
            "in one pass",
}


def main(d="gpurun_out/pmc", out="profiles/pmc_traffic.json", tag="", source="nw"):
    acc = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                name = row.get("Kernel_Name", "?").replace("(anonymous namespace)::", "")
                name = name.split("(")[0].replace("void ", "")
                acc[name][row["Counter_Name"]].append(float(row["Counter_Value"]))
    res = {}
    for k, cs in acc.items():
        if "FETCH_SIZE" not in cs or "WRITE_SIZE" not in cs:
            continue
        fetch = sum(cs["FETCH_SIZE"]) / len(cs["FETCH_SIZE"]) * 1024 * 2
        write = sum(cs["WRITE_SIZE"]) / len(cs["WRITE_SIZE"]) * 1024
        res[k] = {"read_bytes": round(fetch), "write_bytes": round(write),
                  "hbm_bytes": round(fetch + write), "dispatches": len(cs["FETCH_SIZE"])}
        for c, key in (("SQ_INSTS_VALU", "valu_wave_insts"), ("SQ_INSTS_SALU", "salu_wave_insts"),
                       ("SQ_WAVES", "waves"), ("SQ_WAVE_CYCLES", "wave_cycles_q"),
                       ("SQ_BUSY_CYCLES", "busy_cycles_q"), ("SQ_WAIT_INST_ANY", "wait_inst_any_q"),
                       ("SQ_WAIT_ANY", "wait_any_q"), ("SQ_ACTIVE_INST_VALU", "active_inst_valu_q"),
                       ("SQ_ACTIVE_INST_ANY", "active_inst_any_q")):
            if c in cs:  # per-launch means (SQ cycle counters in quad-cycles)
                res[k][key] = round(sum(cs[c]) / len(cs[c]))
        if "SQ_INSTS_VALU" in cs:  # over the whole profiled run (legs: / its executes)
            res[k]["valu_wave_insts_sum"] = round(sum(cs["SQ_INSTS_VALU"]))
            res[k]["valu_dispatches"] = len(cs["SQ_INSTS_VALU"])
        r = res[k]
        if "wave_cycles_q" in r and r["wave_cycles_q"]:
            # shares of the waves' lifetime: issue-stalled on a dependency /
            # parked in s_waitcnt / issuing (disjoint, MI355X_MICROARCH.md SQ row)
            wc = r["wave_cycles_q"]
            for key in ("wait_inst_any_q", "wait_any_q", "active_inst_any_q", "active_inst_valu_q"):
                if key in r:
                    r[key.replace("_q", "_frac")] = round(r[key] / wc, 4)
    doc = {"source": SOURCES.get(source, source), "round": tag, "kernels": res}
    ex = os.path.join(d, "executes.json")  # tools/prof_legs.py
    if os.path.exists(ex):
        with open(ex) as fh:
            doc["executes"] = json.load(fh)
    with open(out, "w") as fh:
        json.dump(doc, fh, indent=1)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:])
