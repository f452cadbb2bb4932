"""configs[2] (C3): WFA with the reference's semantics on 10 kbp G-mut(5%)
pairs, step cap 10^4, through the device-resident WFA plan (sequences and
results in HBM).  n_pairs pairs drawn over `distinct` generated pairs (pair k
uses pair k % distinct).  Reports pairs/s and the status histogram; every
such pair ends in REF_PANIC_TRIM at s = 20.

    python tools/bench_wfa.py [--pairs 1000000] [--distinct 5000] [--reps 3]
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--pairs", type=int, default=1_000_000)
    ap.add_argument("--distinct", type=int, default=5_000)
    ap.add_argument("--len", type=int, default=10_000)
    ap.add_argument("--max-steps", type=int, default=10_000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    import sequencealigning_amd as saln
    from sequencealigning_amd import synth
    seed = 0x5EED0003
    t0 = time.perf_counter()
    allq = synth.random_bases(seed, a.distinct * a.len).tobytes()
    qs = [allq[k * a.len:(k + 1) * a.len] for k in range(a.distinct)]
    ds = [synth.mutate(q, 0.05, seed=k) for k, q in enumerate(qs)]
    q_seq, q_off = saln.pack_csr(qs)
    d_seq, d_off = saln.pack_csr(ds)
    gen_s = time.perf_counter() - t0
    k = np.arange(a.pairs, dtype=np.uint32) % np.uint32(a.distinct)
    t0 = time.perf_counter()
    plan = saln.WfaPlan(q_off, d_off, pairs=np.stack([k, k], 1), max_steps=a.max_steps)
    plan_s = time.perf_counter() - t0
    dq = torch.from_numpy(q_seq.copy()).cuda()
    dd = torch.from_numpy(d_seq.copy()).cuda()
    out = torch.zeros(a.pairs * 8, dtype=torch.int32, device="cuda")
    plan.execute(dq, dd, out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(a.reps):
        plan.execute(dq, dd, out)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / a.reps
    r = out.cpu().numpy().view(saln._lib.WFA_RESULT_DTYPE)
    st, cnt = np.unique(r["status"], return_counts=True)
    print(json.dumps({"workload": f"configs[2]: {a.pairs} WFA pairs ({a.distinct} distinct) of "
                                  f"{a.len} bp G-mut(5%), step cap {a.max_steps}",
                      "pairs": a.pairs, "ms": round(dt * 1e3, 3),
                      "pairs_per_s": round(a.pairs / dt, 1),
                      "status_counts": {saln._lib.STATUS_NAMES.get(int(s), str(int(s))): int(c)
                                        for s, c in zip(st, cnt)},
                      "steps_hist": {int(s): int(c) for s, c in
                                     zip(*np.unique(r["steps"], return_counts=True))},
                      "gen_s": round(gen_s, 2), "plan_s": round(plan_s, 3)}))
    plan.close()


if __name__ == "__main__":
    main()
