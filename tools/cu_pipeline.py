"""C2 fill / walk pipeline on CU partitions (tools only, never
the bench): the configs[1] plan in async mode, execute k's walk on the
plan's traceback stream while execute k+1 fills.  --walk-cus W puts the walk
on W CUs and the fill on the rest (CU-masked streams); --layout picks the
W CUs: "contiguous" mask bits [0, W) (round 3's saln_stream_create_cu_range)
or "balanced" (equal numbers per XCD and shader engine, from
tools/cu_map.py's bit map).  --walk-cus 0: the plain async pipeline (both on
all CUs); --walk-cus -1: sequential steps.  Prints one JSON line; run under
rocprofv3 --kernel-trace for the overlap (tools/trace_overlap.py).

    python tools/cu_pipeline.py --walk-cus 32 --layout balanced --map profiles/r04_cu_map.json
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def balanced_bits(cu_map, w):
    """w mask bits spread evenly over the (XCD, SE) groups of the map."""
    groups = {}
    for b in cu_map["bits"]:
        if len(b["places"]) != 1:
            continue
        x, se = b["places"][0][0], b["places"][0][1]
        groups.setdefault((x, se), []).append(b["bit"])
    keys = sorted(groups)
    if not keys or w > sum(len(v) for v in groups.values()):
        raise SystemExit("cu map has too few single-place bits (re-run tools/cu_map.py)")
    out, r = [], 0
    while len(out) < w:
        for k in keys:
            if r < len(groups[k]) and len(out) < w:
                out.append(groups[k][r])
        r += 1
    return sorted(out)


def mask_stream(L, ctx, bits, ncu):
    words = (C.c_uint32 * ((ncu + 31) // 32))()
    for b in bits:
        words[b // 32] |= 1 << (b % 32)
    h = C.c_void_p()
    rc = L.saln_stream_create_cu_mask(ctx, words, len(words), C.byref(h))
    if rc != 0:
        raise RuntimeError("cu mask stream")
    return h


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--walk-cus", type=int, default=32)
    ap.add_argument("--layout", default="balanced", choices=["contiguous", "balanced"])
    ap.add_argument("--map", default=os.path.join(ROOT, "profiles", "r04_cu_map.json"))
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    a = ap.parse_args()
    import torch
    import sequencealigning_amd as saln
    from sequencealigning_amd import _lib, synth
    L, ctx = _lib.lib(), _lib.context(0)
    n_cu = C.c_uint32()
    _lib.check(L.saln_device_cu_count(ctx, C.byref(n_cu)), "cu_count")
    ncu = n_cu.value
    n, Lq = 100_000, 150
    qs, qo, ds, do = synth.iid_pairs(n, Lq, Lq, seed=0x5EED0002)
    plan = saln.NwPlan(qo, do, pairs=np.stack([np.arange(n), np.arange(n)], 1))
    dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
    res = [torch.zeros(n * 4, dtype=torch.int32, device="cuda") for _ in range(2)]
    cig = [torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda") for _ in range(2)]
    W = a.walk_cus
    fill_s, tb_s, walk_bits = None, None, []
    if W > 0:
        if a.layout == "balanced":
            walk_bits = balanced_bits(json.load(open(a.map)), W)
        else:
            walk_bits = list(range(W))
        fill_bits = [b for b in range(ncu) if b not in set(walk_bits)]
        fill_s = mask_stream(L, ctx, fill_bits, ncu)
        tb_s = mask_stream(L, ctx, walk_bits, ncu)
        _lib.check(L.saln_nw_plan_set_tb_stream(plan._h, tb_s), "set_tb_stream")
    pipelined = W >= 0
    plan.set_async(pipelined)
    stream = fill_s.value if fill_s is not None else None
    state = {"k": 0}

    def step():
        k = state["k"]
        plan.execute(dq, dd, res[k % 2], cig[k % 2], stream=stream)
        state["k"] = k + 1
        if pipelined and k > 0:
            plan.sync(stream=stream, keep_latest=True)

    def drain():
        if pipelined:
            plan.sync(stream=stream)
        torch.cuda.synchronize()
        state["k"] = 0

    for _ in range(a.warmup):
        step()
    drain()
    plan.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        step()
    drain()
    dt = (time.perf_counter() - t0) / a.steps
    plan.check()
    f, fn = plan.kernel_time("nw_fill")
    tb, tn = plan.kernel_time("nw_traceback")
    print(json.dumps({"walk_cus": W, "layout": a.layout if W > 0 else None,
                      "walk_bits": walk_bits[:64], "ms_per_step": round(dt * 1e3, 4),
                      "gcups": round(plan.cells / dt / 1e9, 1),
                      "fill_ms": round(f / max(1, fn), 4), "traceback_ms": round(tb / max(1, tn), 4)}))
    plan.close()
    for h in (fill_s, tb_s):
        if h is not None:
            L.saln_stream_destroy(ctx, h)


if __name__ == "__main__":
    main()
