#!/usr/bin/env python3
"""Headline benchmark: GCUPS of the NW-affine hot path on MI355X.

Headline workload (BASELINE.json configs[1]): 100,000 independent 150 x 150
G-iid DNA pairs per GPU (seed 0x5EED0002 + rank), sequences resident in HBM.
One step = one pass of the hot path over the batch: NW-affine matrix fill
with the 1 B/cell parent mask (nw_fill) + the reference's first-printed
traceback per pair -> score, panic status, CIGAR (nw_traceback); with N > 1
ranks also the RCCL gather of the 16-byte per-pair result records to rank 0
(db sharded).  value = all ranks' cells / max-over-ranks
wall time.

The other BASELINE.json configs ride along as extra keys under "configs"
(SURVEY.md §8(d)), each timed here so the driver's clock covers them, each
with its own `roofline` (the dominant kernel against the HBM or VALU peak)
and `cpu_baseline`:
  c5  configs[4]: 10k x 100k 150 bp score-only all-vs-all, db sharded over
      the N ranks, {score, status} records gathered to rank 0 (every N);
  c1  configs[0]: one 1 kbp pair, GPU latency + the oracle's reference-
      structure CPU path on one core (N = 1);
  c3  configs[2]: WFA (reference semantics) on 10^6 distinct 10 kbp G-mut
      pairs (N = 1);
  c3_affine  the same 10^6 pairs through the corrected gap-affine WFA
      (not reference parity) (N = 1);
  c4  configs[3]: one 100 kbp pair, fill + traceback, + the linear-memory
      oracle on the host cores (N = 1);
  c4_spans  the same pair as 8 column spans (SURVEY.md §8(f) row 3's layout,
      all on this GPU: the band hand-off's cost; 1/8 of the mask per span) (N = 1);
  host_path: configs[1] through the host-buffer C ABI (PCIe-inclusive; never
      the value) (N = 1);
  cli       the drop-in CLI end to end on a 316 x 316-record FASTA of 150 bp
      (batched render, reference text per pair; process wall time) (N = 1).

    python bench.py --gpus N --steps K --warmup W [--legs c2_full,c5,c1,c3,c3_affine,c4,c4_spans,host,cli|none]

With --gpus N > 1 and no WORLD_SIZE in the environment this process starts
the N ranks itself (torch.distributed.run on 127.0.0.1, as a child process;
nothing here touches the GPU first) and exits with their status.  Under an
external launcher WORLD_SIZE must equal --gpus.
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "GCUPS (affine-gap NW) at 1/2/4/8 MI355X; % of HBM roofline"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
# VALU issue peak, MI355X_MICROARCH.md "Wave scheduling": a wave64 VALU op
# issues over 2 cycles on a SIMD-32 -> 1,024 SIMDs x 32 lanes x 2.4 GHz.
VALU_PEAK_TOPS = 1024 * 32 * 2.4e9 / 1e12  # 78.6 T lane-ops/s
# The rate measured for the packed / VOP3 / DPP ops the fill's chain is made
# of (tools/micro/valu_rate.hip: 4 cycles per wave64 op) -> 39.3 T.
VALU_PK_TOPS = 1024 * 16 * 2.4e9 / 1e12
N_PAIRS, LQ, LD = 100_000, 150, 150
SEED = 0x5EED0002
ALL_LEGS = ("c2_full", "c5", "c1", "c3", "c3_affine", "c4", "c4_spans", "host", "cli", "cli_all")
PMC_FILES = ("pmc_traffic.json", "pmc_legs.json", "pmc_c2full.json")  # under profiles/


# SALN_* environment variables the bench runs with (recorded in the JSON
# line).  The engine reads no environment variable (its tuning goes through
# saln_option_set); SALN_LIB would load a tools/ build instead of the
# product, and any other SALN_* is a leftover of an experiment script.
ALLOWED_ENV: tuple = ()


def refused_env(environ=None) -> list:
    environ = os.environ if environ is None else environ
    return sorted(k for k in environ if k.startswith("SALN_") and k not in ALLOWED_ENV)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_threads() -> int:
    """Host threads for the CPU baseline: the box's CPU share (OMP_NUM_THREADS
    is set to it on the GPU pool; os.cpu_count() shows the whole machine)."""
    n = os.cpu_count() or 1
    env = os.environ.get("OMP_NUM_THREADS")
    if env and env.isdigit():
        n = min(n, int(env))
    return max(1, min(n, 16))


# The reference's DFS (needleman_wunsch_affine.rs:281-329) enumerates every
# co-optimal alignment; on 150 x 150 G-iid pairs ~20 % of them need more
# than 10^5 stack pops (round 3 capped there, which overstated the CPU
# path ~4x) and ~1 in 2,000 more than 10^8.  The baseline caps a pair's
# enumeration at 10^8 pops (seconds of CPU) and reports how many hit it.
CPU_MAX_POPS = 100_000_000


def cpu_baseline(budget_s: float = 15.0) -> dict:
    """Oracle (C port of the reference CPU path: full 3-matrix fill with
    parent sets + the reference's exhaustive DFS traceback) on a bounded
    sample of the same workload: one core for ~budget/3 (the reference's own
    sequential loop, main.rs:61-67), then the same port over pairs on all of
    the box's cores for ~2*budget/3."""
    from oracle import refcpu  # cpu_baseline leg only
    from sequencealigning_amd import synth
    refcpu.build()
    n = 60000
    qs, qo, ds, do = synth.iid_pairs(n, LQ, LD, seed=SEED)
    qb, db = qs.tobytes(), ds.tobytes()
    done = cells = capped1 = 0
    t0 = time.perf_counter()
    while done < n and time.perf_counter() - t0 < budget_s / 3:
        k = min(16, n - done)
        c, nc = refcpu.run_pairs_capped(qb[done * LQ:(done + k) * LQ], qo[:k + 1],
                                        db[done * LD:(done + k) * LD], do[:k + 1], k,
                                        max_pops=CPU_MAX_POPS)
        cells += c
        capped1 += nc
        done += k
    dt1 = time.perf_counter() - t0
    rate1 = cells / dt1  # cells/s on one core
    T = cpu_threads()
    # pairs for ~2/3 of the budget at T x the one-core rate (sublinear scaling only shortens it)
    n_mt = int(min(n, max(T * 16, rate1 * T * (2 * budget_s / 3) / (LQ * LD))))
    t0 = time.perf_counter()
    cells_mt, capped_mt = refcpu.run_pairs_capped(qb[:n_mt * LQ], qo[:n_mt + 1], db[:n_mt * LD],
                                                  do[:n_mt + 1], n_mt, max_pops=CPU_MAX_POPS,
                                                  threads=T)
    dtm = time.perf_counter() - t0
    # the round-3 cap on the same multi-core sample, for comparison
    t0 = time.perf_counter()
    cells_5, capped_5 = refcpu.run_pairs_capped(qb[:n_mt * LQ], qo[:n_mt + 1], db[:n_mt * LD],
                                                do[:n_mt + 1], n_mt, max_pops=100_000, threads=T)
    dt5 = time.perf_counter() - t0
    return {"value": round(cells_mt / dtm / 1e9, 6), "unit": "GCUPS", "cores": T, "kind": "port",
            "value_1core": round(rate1 / 1e9, 6),
            "max_pops": CPU_MAX_POPS,
            "capped_pairs": int(capped_mt), "capped_frac": round(capped_mt / max(1, n_mt), 5),
            "capped_pairs_1core": int(capped1),
            "at_1e5_pops": {"value": round(cells_5 / dt5 / 1e9, 6),
                            "capped_frac": round(capped_5 / max(1, n_mt), 4)},
            "sample": f"{n_mt} of the 150x150 G-iid pairs (seed {SEED:#x}) on {T} threads in "
                      f"{dtm:.1f} s, {done} pairs on 1 thread in {dt1:.1f} s; oracle/refcpu.c "
                      f"fill + literal DFS, each pair's enumeration capped at {CPU_MAX_POPS:.0e} "
                      f"stack pops ({capped_mt} of {n_mt} pairs reached it; at round 3's 1e5 "
                      f"cap {capped_5} did)"}


# ------------------------------------------------------------- rooflines
def _pmc_docs(files=PMC_FILES):
    for f in files:
        try:
            with open(os.path.join(ROOT, "profiles", f)) as fh:
                yield f, json.load(fh)
        except (OSError, ValueError):
            continue


def pmc(kernel, field: str = "hbm_bytes", files=PMC_FILES):
    """A per-launch PMC figure of `kernel` (HBM bytes, VALU wave-instructions
    with field="valu_wave_insts", their sum over the profiled run with
    "valu_wave_insts_sum") from the committed PMC summaries (profiles/
    pmc_traffic.json: the headline command; profiles/pmc_legs.json: the
    legs, tools/prof_legs.py), written by tools/pmc_traffic.py from separate
    rocprofv3 --pmc passes (tools/pmc.sh), or None.  `kernel`: a name or a
    tuple of names, the first one found wins; `files`: the summaries to read."""
    for k in ((kernel,) if isinstance(kernel, str) else kernel):
        for _, doc in _pmc_docs(files):
            for name, v in doc.get("kernels", {}).items():
                if k in name and field in v:
                    return v[field]
    return None


def pmc_name(*names: str) -> str:
    """The first of `names` (kernel instantiations a leg may run, e.g. the
    row fill's stripe placements) that the committed PMC summaries hold,
    else the first."""
    return next((k for k in names if pmc(k) is not None), names[0])


def pmc_executes(leg: str):
    """Executes of `leg`'s workload in the profiled run (profiles/pmc_legs.json)."""
    for _, doc in _pmc_docs():
        if leg in doc.get("executes", {}):
            return doc["executes"][leg]
    return None


def roof_hbm(nbytes: float, secs: float, kernel: str, traffic=None, **extra) -> dict:
    """HBM roofline of one kernel launch: algorithmic bytes / its duration."""
    a = nbytes / secs / 1e9
    d = {"bound": "hbm", "achieved": round(a, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
         "frac": round(a / HBM_PEAK_GBS, 5), "traffic": traffic, "kernel": kernel,
         "kernel_avg_ms": round(secs * 1e3, 4), "algorithmic_bytes": int(nbytes)}
    d.update(extra)
    return d


def valu_roof(kernel: str, secs: float, wave_insts=None, **extra):
    """VALU roofline: wave-instructions (PMC SQ_INSTS_VALU from the committed
    summaries) x 64 lanes over the measured duration, against the guide's
    2-cycle wave64 issue peak (78.6 T lane-ops/s); frac_4cycle against the
    4-cycle rate of packed / VOP3 / DPP ops."""
    n = wave_insts if wave_insts is not None else pmc(kernel, "valu_wave_insts")
    if not n:
        return None
    a = n * 64 / secs / 1e12
    d = {"bound": "valu", "achieved": round(a, 3), "peak": round(VALU_PEAK_TOPS, 2),
         "unit": "T int lane-ops/s", "frac": round(a / VALU_PEAK_TOPS, 5),
         "frac_4cycle": round(a / VALU_PK_TOPS, 5), "kernel": kernel,
         "wave_insts": int(n), "seconds": round(secs, 6),
         "source": "SQ_INSTS_VALU from profiles/pmc_*.json (rocprofv3 --pmc of this workload), "
                   "duration measured in this run"}
    d.update(extra)
    return d


def valu_per_execute(kernel: str, leg: str):
    """VALU wave-instructions of one execute of `leg` (all launches of
    `kernel`): the profiled run's sum over its executes."""
    s, ex = pmc(kernel, "valu_wave_insts_sum"), pmc_executes(leg)
    return s / ex if s and ex else None


def verify_c2(res_np, cig_np, cigar_off, qs, qo, ds, do, n_check: int = 1000) -> dict:
    """Untimed check of the benched run's own output: the first n_check
    pairs' score, end states, panic status, printed flag and first printed
    CIGAR against the oracle (oracle/refcheck.c, literal fill + memoised DFS;
    a checker, never the measured path)."""
    from oracle import refcpu  # checker only
    from sequencealigning_amd import _lib
    n = min(n_check, len(qo) - 1)
    want = refcpu.check_pairs(qs[:int(qo[n])], qo[:n + 1], ds[:int(do[n])], do[:n + 1],
                              threads=cpu_threads())
    r = res_np.view(_lib.RESULT_DTYPE)[:n]
    bad = 0
    for k in range(n):
        ok = (int(r["score"][k]) == int(want.score[k])
              and int(r["end_states"][k]) == int(want.end_states[k])
              and (int(r["status"][k]) == _lib.REF_PANIC_BOUNDARY) == bool(want.panics[k])
              and bool(r["printed"][k]) == (want.cig_len[k] >= 0))
        if ok and r["printed"][k]:
            o0 = int(cigar_off[k])
            ok = np.array_equal(cig_np[o0:o0 + int(r["cigar_len"][k])], want.cigar_words(k))
        bad += not ok
    return {"pairs": n, "mismatches": bad, "checker": "oracle/refcheck.c (untimed)"}


def timed(fn, world, dist, torch, local):
    """Barrier + synchronize on both sides; max over ranks of the wall time."""
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    fn()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    dt = time.perf_counter() - t0
    timed.local_s = dt  # this rank's own wall time (rank_diag)
    t = torch.tensor([dt], dtype=torch.float64, device=f"cuda:{local}")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def rank_diag(dist, torch, world: int, device, compute_s: float, gather_s: float,
              gather_bytes: int, wall_s: float | None = None) -> list[dict]:
    """Per-rank diagnosis of a multi-GPU line: every rank's
    compute time, gather time and the bytes its gather moved, all-gathered
    so rank 0 can print them beside the value; a scaling curve then shows
    where its time went (compute imbalance or the RCCL gather)."""
    t = torch.tensor([compute_s, gather_s, float(gather_bytes),
                      -1.0 if wall_s is None else wall_s], dtype=torch.float64, device=device)
    if world > 1:
        out = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(out, t)
    else:
        out = [t]
    rows = []
    for r, x in enumerate(out):
        v = x.cpu().tolist()
        row = {"rank": r, "compute_ms": round(v[0] * 1e3, 3), "gather_ms": round(v[1] * 1e3, 3),
               "gather_bytes": int(v[2])}
        if v[3] >= 0:
            row["wall_ms"] = round(v[3] * 1e3, 3)
        rows.append(row)
    return rows


def gather_probe(dist, torch, world: int, fn, reps: int = 3) -> float:
    """Seconds per call of one gather (fn), untimed by the line: barrier and
    synchronize around each call, min over reps."""
    best = float("inf")
    for _ in range(reps):
        if world > 1:
            dist.barrier()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        best = min(best, time.perf_counter() - t0)
    return best


def event_time(torch, fn, reps: int) -> float:
    """Seconds per call of fn over `reps` calls, from hipEvents on torch's
    current stream (the stream the plans launch on when given none)."""
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    b.synchronize()
    return a.elapsed_time(b) / 1e3 / reps


# ------------------------------------------------------------------- legs
def leg_c5(world, rank, local, dist, torch, nq=10_000, ndb=100_000, L=150, cpu=True):
    """configs[4]: 10k queries x 100k db records of 150 bp (length assumed =
    C2), G-iid (seed 0x5EED0004), score-only all-vs-all with
    the db sharded over the ranks and the records gathered to rank 0
    (dist.ShardedAllVsAll).  Total work is fixed as N grows (strong)."""
    from sequencealigning_amd import _lib, synth
    from sequencealigning_amd.dist import ShardedAllVsAll, shard_db
    seed = 0x5EED0004
    qs = synth.random_bases(seed, nq * L)
    qo = np.arange(nq + 1, dtype=np.uint64) * np.uint64(L)
    do = np.arange(ndb + 1, dtype=np.uint64) * np.uint64(L)
    # every rank draws only its own db block (same stream positions as the full db)
    lo, hi = shard_db(np.full(ndb, L), world, rank)
    ds = np.zeros(ndb * L, np.uint8)
    ds[lo * L:hi * L] = synth.random_bases(seed ^ 0xD5D5D5D5, (hi - lo) * L, start=lo * L)
    t0 = time.perf_counter()
    av = ShardedAllVsAll(qs, qo, ds, do, device=local)
    setup = time.perf_counter() - t0
    av.execute()  # warm: code objects, RCCL communicator
    dt = timed(av.execute, world, dist, torch, local)
    # the fill of this rank's block alone (one launch per query class; events
    # on torch's stream, the stream the engine launches on)
    fill_s = event_time(torch, lambda: av.execute(gather=False, check=False), 1)
    av.check()
    diag = None
    if world > 1:
        g_s = gather_probe(dist, torch, world, av.gather)
        diag = rank_diag(dist, torch, world, f"cuda:{local}", fill_s, g_s,
                         av.cap * 4 * (world if rank == av.dst else 1), wall_s=timed.local_s)
    out = None
    if rank == 0:
        # query profiles (nw.avsa_profile), bonuses in the extension-free frame (nw.pk_tab)
        kern = "nw_fill_avsa_prof_kernel<8, 19, %s>" % (
            "true" if _lib.get_option("nw.pk_tab")[0] else "false")
        ins = valu_per_execute(kern, "c5")
        if ins is not None and world > 1:
            ins *= (hi - lo) / ndb  # this rank's share of the profiled (N = 1) launch
        out = {"workload": f"configs[4]: {nq} x {ndb} score-only all-vs-all, {L} bp G-iid "
                           f"(seed {seed:#x}), db sharded over {world} rank(s), records "
                           f"gathered to rank 0" + (" over RCCL" if world > 1 else ""),
               "value": round(av.cells / dt / 1e9, 1), "unit": "GCUPS", "seconds": round(dt, 4),
               "pairs_per_s": round(nq * ndb / dt, 1), "cells": av.cells, "n_gpus": world,
               "scaling": "strong", "setup_s": round(setup, 2),
               "panic_frac": round(av.status_count(2) / (nq * ndb), 4), "executes": 3,
               "roofline": valu_roof(kern, fill_s, ins, note="score-only: no mask, HBM traffic "
                                     "~0 B/cell; the packed fill's VALU issue is the bound",
                                     gcups_fill=round(av.cells_local / fill_s / 1e9, 1))}
        if diag is not None:
            out["rank_diag"] = {"per_execute": diag,
                                "note": "compute_ms: the rank's block (one execute without the "
                                        "gather, hipEvents); gather_ms: one dist.gather of the "
                                        "{score, status} records to rank 0 (RCCL); gather_bytes: "
                                        "received at rank 0, sent elsewhere"}
        if cpu:
            # checker: a seeded sample of the gathered records against the oracle
            from oracle import refcpu  # checker only
            rng = np.random.default_rng(4)
            di = rng.integers(0, ndb, 256)
            qi = rng.integers(0, nq, 256)
            allq = qs.tobytes()
            dsel = [synth.random_bases(seed ^ 0xD5D5D5D5, L, start=int(d) * L).tobytes() for d in di]
            qsel = [allq[int(q) * L:(int(q) + 1) * L] for q in qi]
            qo2 = np.arange(257, dtype=np.uint64) * np.uint64(L)
            want = refcpu.check_pairs(b"".join(qsel), qo2, b"".join(dsel), qo2,
                                      threads=cpu_threads())
            sc, st = av.lookup(di, qi)
            bad = int(np.sum((sc != want.score) | ((st == 2) != want.panics)))
            out["verified"] = {"pairs": 256, "mismatches": bad,
                               "checker": "oracle/refcheck.c on a seeded sample (untimed)"}
            out["cpu_baseline"] = c5_cpu_baseline(seed, nq, ndb, L)
    av.close()
    del av
    torch.cuda.empty_cache()
    return out


def c5_cpu_baseline(seed, nq, ndb, L, budget_s: float = 8.0) -> dict:
    """The oracle's literal three-matrix fill (oracle/refcpu.c, the reference
    structure; score-only: its DFS stops after one pop) over a seeded slice of
    the C5 pair space on the box's cores, as many pairs as ~budget_s allows."""
    from oracle import refcpu  # cpu_baseline leg only
    from sequencealigning_amd import synth
    T = cpu_threads()
    rng = np.random.default_rng(5)
    allq = synth.random_bases(seed, nq * L)
    n, cells, t_all = 0, 0, 0.0
    chunk = T * 256
    while t_all < budget_s and n < 200_000:
        di = rng.integers(0, ndb, chunk)
        qi = rng.integers(0, nq, chunk)
        dsel = np.concatenate([synth.random_bases(seed ^ 0xD5D5D5D5, L, start=int(d) * L)
                               for d in di]).tobytes()
        qsel = np.concatenate([allq[int(q) * L:(int(q) + 1) * L] for q in qi]).tobytes()
        off = np.arange(chunk + 1, dtype=np.uint64) * np.uint64(L)
        t0 = time.perf_counter()
        cells += refcpu.run_pairs_mt(qsel, off, dsel, off, chunk, max_pops=1, threads=T)
        t_all += time.perf_counter() - t0
        n += chunk
    return {"value": round(cells / t_all / 1e9, 4), "unit": "GCUPS", "cores": T, "kind": "port",
            "seconds": round(t_all, 2),
            "sample": f"{n} pairs drawn from the {nq} x {ndb} pair space (seeded), "
                      f"oracle/refcpu.c literal 3-matrix fill + parent lists (score-only: the DFS "
                      f"stops after one pop) on {T} threads"}


def _single_pair(torch, saln, q, d, reps, score_only=False):
    qo = np.array([0, len(q)], np.uint64)
    do = np.array([0, len(d)], np.uint64)
    plan = saln.NwPlan(qo, do, pairs=[(0, 0)])
    plan.set_score_only(score_only)
    dq = torch.frombuffer(bytearray(q), dtype=torch.uint8).cuda()
    dd = torch.frombuffer(bytearray(d), dtype=torch.uint8).cuda()
    res = torch.zeros(4, dtype=torch.int32, device="cuda")
    cig = torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
    plan.execute(dq, dd, res, cig)
    torch.cuda.synchronize()
    plan.set_timing(True)
    t0 = time.perf_counter()
    for _ in range(reps):
        plan.execute(dq, dd, res, cig)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    plan.check()  # a column-stripe dependency timeout raises here
    f, _ = plan.kernel_time("nw_fill")
    tb, _ = plan.kernel_time("nw_traceback")
    r = res.cpu().numpy().view(saln._lib.RESULT_DTYPE)[0]
    words = cig.cpu().numpy().view(np.uint32)[:int(r["cigar_len"])]
    ops = saln.cigar_ops_string(saln.nw._decode_cigar(words)) if r["printed"] else None
    out = {"len_q": len(q), "len_db": len(d), "cells": plan.cells, "score": int(r["score"]),
           "status": int(r["status"]), "printed": int(r["printed"]), "flags": int(r["flags"]),
           "execute_ms": round(dt * 1e3, 4), "fill_ms": round(f / reps, 4),
           "traceback_ms": round(tb / reps, 4), "gcups": round(plan.cells / dt / 1e9, 2)}
    plan.close()
    return out, ops


def leg_c1(torch, saln, reps=50, cpu=True):
    """configs[0]: one 1 kbp x 1 kbp pair (G-mut 5 %, seed 0x5EED0000; and a
    G-iid pair), score + first-printed traceback on the GPU, next to the
    reference-structure CPU path on one core (the oracle's literal fill +
    DFS that prints every co-optimal alignment, needleman_wunsch_affine.rs
    :424-437)."""
    from sequencealigning_amd import synth
    q = synth.random_bases(0x5EED0000, 1000).tobytes()
    d = synth.mutate(q, 0.05, seed=1000)
    gi = synth.random_bases(0x5EED0000 ^ 0x77, 1000).tobytes()
    g, ops = _single_pair(torch, saln, q, d, reps)
    g_iid, ops_iid = _single_pair(torch, saln, q, gi, reps)
    # 16 stripes, one per SIMD (kPlace 2: XCD-local runs on a whole-device stream; 1: lone)
    kern = pmc_name("nw_fill_rows_kernel<1, 0, true, 2>", "nw_fill_rows_kernel<1, 0, true, 1>")
    fill_s = g["fill_ms"] / 1e3
    out = {"workload": "configs[0]: one 1 kbp x 1 kbp pair, score + first-printed traceback "
                       "(G-mut 5 %; iid beside it)",
           "gpu": g, "gpu_iid": g_iid, "executes": 2 * (1 + reps),
           "roofline": roof_hbm(g["cells"], fill_s, kern, pmc(kern),
                                note="latency-bound: one pair's 998-row chain through 16 "
                                     "64-column stripes (1,024 SIMDs, 16 waves)",
                                valu=valu_roof(kern, fill_s, valu_per_execute(kern, "c1")))}
    if not cpu:
        return out
    from oracle import refcpu  # cpu_baseline leg only
    qo = np.array([0, len(q)], np.uint64)
    do = np.array([0, len(d)], np.uint64)
    n, t0 = 0, time.perf_counter()
    while n < 3 or time.perf_counter() - t0 < 2.0:
        refcpu.run_pairs(q, qo, d, do, 1, max_pops=10_000_000)
        n += 1
    cpu_s = (time.perf_counter() - t0) / n
    o = refcpu.nw(q, d, literal_dfs=False)
    oi = refcpu.nw(q, gi, literal_dfs=False)
    out["cpu_baseline"] = {"ms": round(cpu_s * 1e3, 3), "cores": 1, "kind": "port",
                           "gcups": round(len(q) * len(d) / cpu_s / 1e9, 5),
                           "sample": f"the same pair, {n} runs of oracle/refcpu.c fill + "
                                     "literal DFS (every co-optimal block)"}
    out["matches_oracle"] = bool(
        g["score"] == o.score and (g["status"] == 2) == o.panics and ops == o.first_ops
        and g_iid["score"] == oi.score and (g_iid["status"] == 2) == oi.panics
        and ops_iid == oi.first_ops)
    out["checked"] = "score, panic status and the first printed CIGAR of both pairs"
    out["speedup_vs_cpu"] = round(cpu_s * 1e3 / g["execute_ms"], 1)
    return out


def leg_c2_full(torch, saln, n=N_PAIRS, steps=10, warmup=2):
    """configs[1] as SURVEY 8(d) defines it: 10^5 G-iid 150x150 pairs, fill +
    the reference's full parent sets stored (1 B/cell, the 7 parent bits of
    needleman_wunsch_affine.rs:96-153 that the all-blocks DFS :281-329 reads;
    saln_nw_plan_create_full) + the first printed traceback / CIGAR (the
    headline stores 4-bit walk codes instead).  Sequential steps, fill then
    walk: beside the next fill the full-code walk (a lane per pair) costs the
    fill more than it overlaps (round 6, profiles/r06_full_tab_ab.jsonl:
    1.353-1.356 ms per step sequential, 1.367-1.376 pipelined)."""
    from sequencealigning_amd import synth
    qs, qo, ds, do = synth.iid_pairs(n, LQ, LD, seed=SEED)
    plan = saln.NwPlan(qo, do, pairs=np.stack([np.arange(n), np.arange(n)], 1), full_codes=True)
    dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
    res = [torch.zeros(n * 4, dtype=torch.int32, device="cuda") for _ in range(2)]
    cig = [torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
           for _ in range(2)]
    for k in range(warmup):
        plan.execute(dq, dd, res[k % 2], cig[k % 2])
    torch.cuda.synchronize()
    plan.set_timing(True)
    t0 = time.perf_counter()
    for k in range(steps):
        plan.execute(dq, dd, res[k % 2], cig[k % 2])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / steps
    plan.check()
    fill_ms, fill_n = plan.kernel_time("nw_fill")
    tb_ms, tb_n = plan.kernel_time("nw_traceback")
    last = (steps - 1) % 2
    hr = res[last].cpu().numpy()
    verified = verify_c2(hr, cig[last].cpu().numpy().view(np.uint32), plan.cigar_off, qs, qo, ds,
                         do)
    fa_ms, fa_n = fill_ms, fill_n  # every fill of a sequential plan runs alone
    # the dense parent sets of one pair of the timed plan, against the oracle (untimed)
    from oracle import refcpu  # checker only
    mask_ok = all(np.array_equal(plan.dense_mask(k), refcpu.nw(
        qs[qo[k]:qo[k + 1]].tobytes(), ds[do[k]:do[k + 1]].tobytes(),
        literal_dfs=False).dense_mask) for k in (0, n // 2, n - 1))
    cells = plan.cells
    plan.close()
    fill_s, alone_s = fill_ms / max(1, fill_n) / 1e3, fa_ms / max(1, fa_n) / 1e3
    # the table fill with row profiles (round 6; nw.pk_tab), else the generic one
    kern = pmc_name("nw_fill_pk_tab_kernel<16, 10, saln::PlanSrc, 3, 1>",
                    "nw_fill_pk_kernel<16, 10, 1, saln::PlanSrc, 10, false>")
    return {"workload": "configs[1] as SURVEY 8(d) defines it: 10^5 independent 150x150 G-iid "
                        "pairs, fill + full 1 B/cell parent sets (7 bits: argmax {M,I,D}, I and "
                        "D extend/open) + first-printed traceback/CIGAR, sequential steps",
            "value": round(cells / dt / 1e9, 2), "unit": "GCUPS", "ms_per_step": round(dt * 1e3, 4),
            "steps": steps, "cells": cells, "executes": warmup + steps, "pipelined": False,
            "roofline": roof_hbm(cells, fill_s, kern, pmc(kern),
                                 kernel_avg_ms_alone=round(alone_s * 1e3, 4),
                                 frac_alone=round(cells / alone_s / 1e9 / HBM_PEAK_GBS, 4),
                                 step_frac=round(cells / dt / 1e9 / HBM_PEAK_GBS, 4),
                                 traceback_avg_ms=round(tb_ms / max(1, tb_n), 4),
                                 note="algorithmic bytes = 1 B/cell, here also the bytes the "
                                      "fill stores; traffic from profiles/pmc_c2full.json",
                                 valu=valu_roof(kern, fill_s)),
            "verified": verified, "dense_mask_equal_oracle": bool(mask_ok),
            "cpu_baseline": "the headline's (the oracle's fill computes every parent set)"}


def leg_c4(torch, saln, reps=3, cpu=True):
    """configs[3]: one 100 kbp x 100 kbp pair (G-mut 5 %, seed 0x5EED0003),
    fill + parent mask + first-printed traceback on one GPU, and the
    linear-memory oracle (reflinear.c: column stripes on the host cores,
    1 B of parent sets per cell, the reference DFS's first event) on the same
    pair for score + CIGAR parity and the CPU time."""
    from sequencealigning_amd import synth
    q = synth.random_bases(0x5EED0003, 100_000).tobytes()
    d = synth.mutate(q, 0.05, seed=100_000)
    g, ops = _single_pair(torch, saln, q, d, reps)
    torch.cuda.empty_cache()
    # 782 stripes, one per SIMD, XCD-local runs (nw.rows_xcd)
    kern = pmc_name("nw_fill_rows_kernel<2, 0, true, 2>", "nw_fill_rows_kernel<2, 0, true, 1>")
    fill_s = g["fill_ms"] / 1e3
    out = {"workload": "configs[3]: one 100 kbp x 100 kbp pair, G-mut 5 %, fill + 1 B/cell mask "
                       "+ first-printed traceback", "gpu": g, "executes": 1 + reps,
           "value": g["gcups"], "unit": "GCUPS",
           "roofline": roof_hbm(g["cells"], fill_s, kern, pmc(kern),
                                note="bound by the 100,001-row chain of lone stripe waves "
                                     "(DESIGN.md §3), not by HBM",
                                valu=valu_roof(kern, fill_s, valu_per_execute(kern, "c4")))}
    if not cpu:
        return out
    from oracle import refcpu  # cpu_baseline leg only
    T = cpu_threads()
    t0 = time.perf_counter()
    sc, es, pan, first, _ = refcpu.nw_first_linear(q, d, threads=T)
    cpu_s = time.perf_counter() - t0
    out["matches_oracle"] = bool(g["score"] == sc and (g["status"] == 2) == pan and ops == first)
    out["checked"] = "score, panic status and the first printed CIGAR (~101k ops)"
    out["cpu_baseline"] = {"seconds": round(cpu_s, 2), "cores": T, "kind": "port",
                           "gcups": round(len(q) * len(d) / cpu_s / 1e9, 3),
                           "sample": "the whole pair, oracle/reflinear.c: linear-memory fill "
                                     "keeping 1 B of parent sets per cell + the reference DFS's "
                                     "first alignment (the reference-structure path needs ~TB)"}
    return out


def leg_c4_spans(torch, saln, n_spans=8, reps=3, band_rows=1024, edge_masks="shared",
                 cu_ranges=None):
    """configs[3]'s pair split by query columns into `n_spans` spans
    (span.py SpanChain): the spans' fills run
    concurrently on this GPU, each on its own slice of the CUs, and a relay
    kernel per edge hands each boundary row over as it is published; then the
    walk crosses the spans right to left.  The 8-GPU layout on one GPU: each span keeps 1/8 of the
    mask, the stripes are 128 columns wide (the whole pair's stripes share
    this GPU's SIMDs) and the time is the hand-off protocol's cost over the
    one-plan fill (c4); span_fill_alone_ms: each span alone with 64-column
    stripes, as on a GPU of its own.  Checked word for word against the plan
    path (n_w_align)."""
    from sequencealigning_amd import synth
    from sequencealigning_amd.span import SpanChain
    q = synth.random_bases(0x5EED0003, 100_000).tobytes()
    d = synth.mutate(q, 0.05, seed=100_000)
    ch = SpanChain(q, d, n_spans, band_rows=band_rows, edge_masks=edge_masks, cu_ranges=cu_ranges)
    fills, walks, r = [], [], None
    for k in range(1 + reps):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ch.fill(pipelined=True)
        torch.cuda.synchronize()
        t1 = time.perf_counter()
        r = ch.walk()
        t2 = time.perf_counter()
        if k:
            fills.append(t1 - t0)
            walks.append(t2 - t1)
    # each span alone on the GPU with the stripe width of a GPU that holds
    # only it (its inbox the chain's boundary): the fill time of one GPU of an
    # n_spans-GPU node
    from sequencealigning_amd.span import NwSpan
    main = torch.cuda.current_stream()
    alone = []
    for k_s, (lo, hi) in enumerate(ch.cols):
        sp = NwSpan(len(q), len(d), lo, hi, device=torch.cuda.current_device())
        ms = []
        for k in range(2):
            sp.reset(main)
            if k_s:
                sp.inbox.copy_(ch.spans[k_s - 1].outbox)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record(main)
            sp.fill(ch.q, ch.d, main)
            e1.record(main)
            torch.cuda.synchronize()
            sp.check()
            ms.append(e0.elapsed_time(e1))
        alone.append(ms[-1])
        sp.close()
    span_mask = max(s.mask_bytes for s in ch.spans)
    ch.close()
    torch.cuda.empty_cache()
    want = saln.n_w_align(q, d)
    fill_s, walk_s = float(np.mean(fills)), float(np.mean(walks))
    cells = len(q) * len(d)
    # the chain's span fills (128-column stripes on CU-masked streams, one
    # per SIMD of the span's CUs, in XCD runs when they fit), one launch per
    # span and execute; their own PMC summary (tools/prof_legs.py c4_spans:
    # the same instantiation as the c4 leg's fill)
    span_kern = "nw_fill_rows_kernel<2, 0, true,"
    per_launch = pmc(span_kern, files=("pmc_c4_spans.json",))
    span_traffic = per_launch * n_spans if per_launch else None
    return {"workload": f"configs[3]'s pair as {n_spans} column spans on one GPU, each on "
                        f"1/{n_spans} of its CUs (CU-masked streams), boundary rows relayed "
                        f"span to span as they are published (one relay kernel per edge)", "value": round(cells / (fill_s + walk_s) / 1e9, 1),
            "unit": "GCUPS", "fill_ms": round(fill_s * 1e3, 3), "walk_ms": round(walk_s * 1e3, 3),
            "walk_ms_reps": [round(x * 1e3, 3) for x in walks],
            "executes": 1 + reps + 2, "span_fill_alone_ms": [round(x, 3) for x in alone],
            "mask_bytes_per_span": int(span_mask),
            "mask_bytes_pair": cells,
            "matches_plan": bool((r.score, r.status, r.end_states, r.printed, r.cigar) ==
                                 (want.score, want.status, want.end_states, want.printed,
                                  want.cigar)),
            "checked": "score, status, end states and the first printed CIGAR vs n_w_align",
            "roofline": roof_hbm(cells, fill_s, "nw_fill_rows_kernel (8 spans, CU-partitioned)",
                                 span_traffic, traffic_kernel=span_kern,
                                 note="1 B/cell of mask over the spans' concurrent fills; bound "
                                      "by the row chain like c4 (DESIGN.md §6); traffic: the "
                                      "spans' fill launches of one execute (PMC, "
                                      "profiles/pmc_c4_spans.json)"),
            "cpu_baseline": "the c4 leg's (the same pair)"}


_C3_PAIRS = {}


def leg_c4_sharded(world, rank, local, dist, torch, reps=3, band_rows=1024, engine=None,
                   q=None, d=None):
    """SURVEY 8(f) row 3 at N > 1: configs[3]'s pair (100 kbp x 100 kbp G-mut
    5 %, seed 0x5EED0003) split by query columns over the ranks, one span
    per GPU (span.ShardedLongPair: the boundary rows travel rank r -> r+1 in
    bands over RCCL send/recv while the spans fill, then the walk crosses the
    ranks right to left and rank 0 assembles the CIGAR; main.rs:61-62 runs
    the pair on one core).  Every rank returns the line; rank 0's holds
    per-rank fill / walk / wall times and a probe of the band exchange alone
    (the whole boundary column sent r -> r+1 in bands, after the timed runs).
    engine / q / d: a CPU span engine and a small pair (tests, gloo)."""
    import numpy as _np

    from sequencealigning_amd.span import ShardedLongPair
    if q is None:
        from sequencealigning_amd import synth
        q = synth.random_bases(0x5EED0003, 100_000).tobytes()
        d = synth.mutate(q, 0.05, seed=100_000)
    on_gpu = engine is None
    sync = (lambda: torch.cuda.synchronize(local)) if on_gpu else (lambda: None)
    sp = ShardedLongPair(q, d, band_rows=band_rows, engine=engine)
    lo, hi = sp.cols[rank]
    fills, walks, walls = [], [], []
    res = None
    for it in range(1 + reps):  # the first run warms up (not timed)
        dist.barrier()
        sync()
        t0 = time.perf_counter()
        sp.fill()
        sync()
        t1 = time.perf_counter()
        res = sp.walk()
        sync()
        t2 = time.perf_counter()
        if it:
            fills.append(t1 - t0)
            walks.append(t2 - t1)
            walls.append(t2 - t0)
    # the band exchange alone: every band of the boundary column r -> r+1
    tdev = torch.device("cuda", local) if on_gpu and sp.nccl else torch.device("cpu")
    dist.barrier()
    sync()
    t0 = time.perf_counter()
    for a, b in sp.bands:
        buf = torch.zeros(b - a + 1, dtype=torch.int64, device=tdev)
        if sp.left is not None:
            dist.recv(buf, src=rank - 1, group=sp.left)
        if sp.right is not None:
            dist.send(buf, dst=rank + 1, group=sp.right)
    sync()
    band_s = time.perf_counter() - t0
    sp.close()
    mine = _np.array([rank, hi - lo, _np.median(fills) * 1e3, _np.median(walks) * 1e3,
                      _np.median(walls) * 1e3, band_s * 1e3], _np.float64)
    t = torch.tensor(mine, dtype=torch.float64, device=tdev)
    parts = [torch.zeros_like(t) for _ in range(world)] if rank == 0 else None
    dist.gather(t, parts, dst=0)
    wall_max = torch.tensor([max(walls)], dtype=torch.float64, device=tdev)
    dist.all_reduce(wall_max, op=dist.ReduceOp.MAX)
    if rank != 0:
        return {}
    per = [dict(zip(("rank", "cols", "fill_ms", "walk_ms", "wall_ms", "band_exchange_ms"),
                    [int(x[0]), int(x[1])] + [round(float(v), 3) for v in x[2:]]))
           for x in (p.cpu().numpy() for p in parts)]
    cells = len(q) * len(d)
    med = float(_np.median([max(p["wall_ms"] for p in per)]))
    return {"workload": f"configs[3]'s pair ({len(q)} x {len(d)}) as {world} column spans, one "
                        f"per rank (ShardedLongPair: {band_rows}-row bands over "
                        f"{'RCCL' if sp.nccl else 'the host relay'}, right-to-left walk, CIGAR "
                        f"on rank 0)",
            "value": round(cells / (med / 1e3) / 1e9, 5), "unit": "GCUPS",
            "ms": round(med, 3), "ms_max": round(float(wall_max.item()) * 1e3, 3),
            "n_ranks": world, "reps": reps, "per_rank": per,
            "result": {"score": int(res.score), "status": int(res.status),
                       "printed": int(res.printed), "cigar_runs": len(res.cigar)},
            "note": "value: cells / the slowest rank's median fill + walk; fill_ms includes "
                    "the waits for the left neighbour's bands; band_exchange_ms: the whole "
                    "boundary column sent r -> r+1 band by band, alone, after the timed runs"}


def c3_pairs(torch, n_pairs, L):
    """configs[2]'s 10^6 distinct 10 kbp G-mut(5 %) pairs, generated on the
    device once (synth.mut_pairs_torch) and shared by c3 and c3_affine."""
    from sequencealigning_amd import synth
    key = (n_pairs, L)
    if key not in _C3_PAIRS:
        _C3_PAIRS.clear()
        t0 = time.perf_counter()
        p = synth.mut_pairs_torch(n_pairs, L, 0.05, 0x5EED0003, "cuda")
        torch.cuda.synchronize()
        _C3_PAIRS[key] = p + (time.perf_counter() - t0,)
    return _C3_PAIRS[key]


def leg_c3(torch, saln, n_pairs=1_000_000, L=10_000, reps=3, cpu=True):
    """configs[2]: WFA with the reference's semantics (wfa.rs) on 10^6
    distinct 10 kbp G-mut(5 %) pairs generated on the device, step cap 10^4,
    sequences and results in HBM."""
    qs, qo, ds, do, gen_s = c3_pairs(torch, n_pairs, L)
    k = np.arange(n_pairs, dtype=np.uint32)
    plan = saln.WfaPlan(qo, do, pairs=np.stack([k, k], 1), max_steps=10_000)
    out_t = torch.zeros(n_pairs * 8, dtype=torch.int32, device="cuda")
    plan.execute(qs, ds, out_t)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        plan.execute(qs, ds, out_t)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / reps
    ev_s = event_time(torch, lambda: plan.execute(qs, ds, out_t), 1)
    r = out_t.cpu().numpy().view(saln._lib.WFA_RESULT_DTYPE)
    st, cnt = np.unique(r["status"], return_counts=True)
    kern = "wfa_kernel"
    out = {"workload": f"configs[2]: {n_pairs} distinct WFA pairs of {L} bp G-mut(5 %), "
                       "reference semantics, step cap 1e4",
           "value": round(n_pairs / dt, 1), "unit": "pairs/s", "ms": round(dt * 1e3, 3),
           "status_counts": {saln._lib.STATUS_NAMES.get(int(s), str(int(s))): int(c)
                             for s, c in zip(st, cnt)},
           "gen_s": round(gen_s, 2), "executes": 2 + reps,
           "roofline": valu_roof(kern, ev_s, valu_per_execute(kern, "c3"),
                                 note="every pair ends in REF_PANIC_TRIM at s = 20 (wfa.rs:603): "
                                      "20 score steps of one lane per pair")}
    if cpu:
        from oracle import refcpu  # cpu_baseline leg only
        samp = np.random.default_rng(3).choice(n_pairs, 200, replace=False)
        bad, t0 = 0, time.perf_counter()
        for p in samp:
            qq = qs[int(qo[p]):int(qo[p + 1])].cpu().numpy().tobytes()
            dd = ds[int(do[p]):int(do[p + 1])].cpu().numpy().tobytes()
            o = refcpu.wfa(qq, dd, max_steps=10_000)
            rr = r[p]
            bad += not (int(rr["status"]) == o.status and int(rr["score"]) == o.score
                        and int(rr["steps"]) == o.steps)
        cpu_s = (time.perf_counter() - t0) / len(samp)
        out["verified"] = {"pairs": len(samp), "mismatches": bad,
                           "checker": "oracle/refwfa.c status, printed score, steps (untimed)"}
        out["cpu_baseline"] = {"pairs_per_s": round(1 / cpu_s, 1), "cores": 1, "kind": "port",
                               "sample": f"{len(samp)} of the pairs through oracle/refwfa.c "
                                         "(its stdout text included)"}
    plan.close()
    del out_t
    torch.cuda.empty_cache()
    return out


def leg_c3_affine(torch, saln, n_pairs=1_000_000, L=10_000, reps=1, cpu=True):
    """configs[2]'s pairs through the corrected gap-affine WFA (SURVEY.md
    §8(f) row 4; not reference parity): the minimum penalty with wfa.rs:14-21's
    x = 4, o = 2, e = 6, sequences and scores in HBM.  A seeded sample of 200
    pairs is checked against the Gotoh DP (oracle/refaffine.c), which is also
    the CPU baseline (on the box's cores)."""
    from sequencealigning_amd.wfa_affine import WfaAffinePlan
    qs, qo, ds, do, gen_s = c3_pairs(torch, n_pairs, L)
    k = np.arange(n_pairs, dtype=np.uint32)
    plan = WfaAffinePlan(qo, do, np.stack([k, k], 1))
    sc = torch.zeros(n_pairs, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    ev_s = event_time(torch, lambda: plan.execute(qs, ds, sc), reps)
    dt = (time.perf_counter() - t0) / reps
    s = sc.cpu().numpy()
    kern = "wfa_affine_kernel"
    out = {"workload": f"configs[2] pairs ({n_pairs} distinct, {L} bp G-mut 5 %) through the "
                       "corrected gap-affine WFA (x=4, o=2, e=6; score only; not reference parity)",
           "value": round(n_pairs / dt, 1), "unit": "pairs/s", "seconds": round(dt, 3),
           "penalty_mean": round(float(s[s >= 0].mean()), 1) if (s >= 0).any() else None,
           "over_limits": int((s < 0).sum()), "executes": reps,
           "roofline": valu_roof(kern, ev_s, valu_per_execute(kern, "c3_affine"),
                                 note="one wave per pair over diagonal groups of 4 x 64 lanes; "
                                      "issue and LDS latency (DESIGN.md §3b)")}
    if cpu:
        from oracle import refcpu  # checker + cpu_baseline only
        samp = np.sort(np.random.default_rng(6).choice(n_pairs, 200, replace=False))
        qh = np.concatenate([qs[int(qo[p]):int(qo[p + 1])].cpu().numpy() for p in samp])
        dh = np.concatenate([ds[int(do[p]):int(do[p + 1])].cpu().numpy() for p in samp])
        ql = np.array([int(qo[p + 1] - qo[p]) for p in samp], np.uint64)
        dl = np.array([int(do[p + 1] - do[p]) for p in samp], np.uint64)
        qo2 = np.concatenate([[0], np.cumsum(ql)]).astype(np.uint64)
        do2 = np.concatenate([[0], np.cumsum(dl)]).astype(np.uint64)
        idx = np.arange(len(samp), dtype=np.uint32)
        T = cpu_threads()
        t0 = time.perf_counter()
        want = refcpu.affine_run_pairs(qh, qo2, dh, do2, idx, idx, threads=T)
        cpu_s = time.perf_counter() - t0
        out["verified"] = {"pairs": len(samp), "mismatches": int(np.sum(want != s[samp])),
                           "checker": "oracle/refaffine.c Gotoh DP (untimed)"}
        out["cpu_baseline"] = {"pairs_per_s": round(len(samp) / cpu_s, 2), "cores": T,
                               "kind": "port", "seconds": round(cpu_s, 2),
                               "sample": f"{len(samp)} of the pairs through oracle/refaffine.c "
                                         f"(O(n*m) Gotoh DP) on {T} threads"}
    plan.close()
    del sc
    torch.cuda.empty_cache()
    return out


def leg_host(saln):
    """configs[1] through the host-buffer boundary (saln_nw_align_batch):
    plan + H2D + fill + traceback + D2H of results and CIGARs.  The
    PCIe-inclusive rate a caller with host arrays sees; never the value."""
    import ctypes as C

    from sequencealigning_amd import _lib, synth
    n = N_PAIRS
    qs, qo, ds, do = synth.iid_pairs(n, LQ, LD, seed=SEED)
    pq = np.arange(n, dtype=np.uint32)
    res = np.zeros(n, dtype=_lib.RESULT_DTYPE)
    coff = np.zeros(n + 1, np.uint64)
    coff[1:] = np.cumsum(np.full(n, LQ + LD, np.uint64))
    cig = np.zeros(int(coff[-1]), np.uint32)
    vp = lambda x: x.ctypes.data_as(C.c_void_p)  # noqa: E731
    L, ctx = _lib.lib(), _lib.context(0)

    def run():
        _lib.check(L.saln_nw_align_batch(ctx, vp(qs), vp(qo), n, vp(ds), vp(do), n,
                                         vp(pq), vp(pq), n, 0, None, vp(res), vp(cig),
                                         vp(coff)), "saln_nw_align_batch")
    run()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        run()
    dt = (time.perf_counter() - t0) / reps
    return {"workload": f"configs[1] via saln_nw_align_batch (host buffers): {n} 150x150 pairs",
            "value": round(n * LQ * LD / dt / 1e9, 1), "unit": "GCUPS (PCIe-inclusive)",
            "ms": round(dt * 1e3, 2)}


def leg_cli(saln, n: int = 316, cpu: bool = True, max_blocks: int = 1, gmut: bool = False) -> dict:
    """The drop-in CLI end to end (`saln -q Q.fa -d D.fa -a needleman-wunsch`,
    main.rs:19-80) on n x n FASTA records of 150 bp, every pair computed once
    in render batches (saln_nw_render_batch), each pair's reference text
    printed; --no-abort: every pair, where the reference would stop at the
    first panic; --no-timing: no nondeterministic lines.
    - default (`cli`): G-iid records (seed 0x5EED0002; ~configs[1]'s 10^5
      pairs), --max-blocks 1 (the first block, so the stdout stays bounded);
    - gmut (`cli_all`): every record a G-mut(5 %) copy of one 150 bp base, so
      each pair is ~10 % divergent with a few to thousands of co-optimal
      alignments, and the reference's default output: every block
      (max_blocks 0), the host DFS over the GPU's parent codes.
    Wall time of the process, FASTA parse and context creation included.  The
    first n pairs of stdout are checked against the oracle's literal DFS text;
    the CPU baseline is the oracle's fill + DFS (same block cap) over every
    pair of the file."""
    import subprocess
    import tempfile

    from sequencealigning_amd import synth
    cli = os.path.join(ROOT, "sequencealigning_amd", "saln")
    if gmut:
        rng = np.random.default_rng(SEED)
        base = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), LQ))
        q = [synth.mutate(base, 0.05, seed=SEED + k) for k in range(n)]
        d = [synth.mutate(base, 0.05, seed=SEED + n + k) for k in range(n)]
        qs, ds = np.frombuffer(b"".join(q), np.uint8), np.frombuffer(b"".join(d), np.uint8)
        qo = np.concatenate([[0], np.cumsum([len(x) for x in q])]).astype(np.uint64)
        do = np.concatenate([[0], np.cumsum([len(x) for x in d])]).astype(np.uint64)
        kind = f"G-mut(5 %) copies of one {LQ} bp base"
    else:
        qs, qo, ds, do = synth.iid_pairs(n, LQ, LD, seed=SEED)
        q = [qs[int(qo[k]):int(qo[k + 1])].tobytes() for k in range(n)]
        d = [ds[int(do[k]):int(do[k + 1])].tobytes() for k in range(n)]
        kind = f"{LQ} bp G-iid"
    with tempfile.TemporaryDirectory() as tdir:
        qf, df, of = (os.path.join(tdir, x) for x in ("q.fa", "d.fa", "out.txt"))
        for path, recs, tag in ((qf, q, "q"), (df, d, "d")):
            with open(path, "wb") as fh:
                for k, r in enumerate(recs):
                    fh.write(b">%s%d\n%s\n" % (tag.encode(), k, r))
        cmd = [cli, "-q", qf, "-d", df, "-a", "needleman-wunsch", "--no-timing", "--no-abort"]
        if max_blocks:
            cmd += ["--max-blocks", str(max_blocks)]
        walls = []
        # timed runs write the text to /dev/null, like the CPU baseline below
        # (both format every byte; neither pays for a file system)
        for k in range(6):  # the first run also pages in the library; value: the median of 5
            with open(os.devnull, "wb") as out:
                t0 = time.perf_counter()
                r = subprocess.run(cmd, stdout=out, stderr=subprocess.PIPE, timeout=600)
                walls.append(time.perf_counter() - t0)
            if r.returncode != 0:
                raise RuntimeError(f"saln exited {r.returncode}: {r.stderr[-500:]!r}")
        # one more run into a file: the text checked below, and its stage
        # breakdown (stderr; not the timed value)
        with open(of, "wb") as out:
            t0 = time.perf_counter()
            r = subprocess.run(cmd + ["--stage-times"], stdout=out, stderr=subprocess.PIPE,
                               timeout=600)
            wall_file = time.perf_counter() - t0
        if r.returncode != 0:
            raise RuntimeError(f"saln exited {r.returncode}: {r.stderr[-500:]!r}")
        stages = [ln.split("]", 1)[1].strip() for ln in r.stderr.decode("latin-1").splitlines()
                  if ln.startswith("[saln ")]
        with open(of, "rb") as fh:
            head = fh.read(64 << 20).decode("latin-1")
        out_bytes = os.path.getsize(of)
        os.remove(of)
    from oracle import refcpu  # untimed checker / cpu baseline only
    want = "".join(refcpu.nw(a, d[0], max_blocks=max_blocks, max_pops=CPU_MAX_POPS,
                             out_cap=1 << 26).stdout for a in q)
    lq, ld = np.diff(qo).astype(np.int64), np.diff(do).astype(np.int64)
    cells = int(lq.sum() * ld.sum())
    flags = "--no-timing --no-abort" + (f" --max-blocks {max_blocks}" if max_blocks else "")
    res = {"workload": f"saln CLI (-a needleman-wunsch {flags}) on {n} x {n} FASTA records, "
                       f"{kind} ({n * n} pairs, seed {SEED:#x})",
           "value": round(cells / float(np.median(walls[1:])) / 1e9, 2),
           "unit": "GCUPS (process wall time, stdout to /dev/null, median of 5 runs after a "
                   "first)",
           "stages_ms": stages, "wall_s_to_file": round(wall_file, 3),
           "wall_s": round(float(np.median(walls[1:])), 3), "wall_s_first": round(walls[0], 3),
           "walls_s": [round(w, 3) for w in walls],
           "stdout_bytes": out_bytes,
           "verified": {"pairs": n, "match": head.startswith(want),
                        "checker": "oracle/refcpu.c literal DFS text, first db record x every "
                                   "query (untimed)"}}
    if cpu:
        T = cpu_threads()
        # every pair of the file (db outer, query inner), on T threads
        m = n * n
        qi, di = np.arange(m) % n, np.arange(m) // n
        sq = b"".join(q[i] for i in qi)
        sd = b"".join(d[j] for j in di)
        qoff = np.concatenate([[0], np.cumsum(lq[qi])]).astype(np.uint64)
        doff = np.concatenate([[0], np.cumsum(ld[di])]).astype(np.uint64)
        blk = (f"stopped before block {max_blocks + 1}" if max_blocks else "over every block")
        # text-inclusive: every pair's reference text formatted and written to
        # /dev/null in pair order (oracle/refmt.c ref_nw_run_pairs_text_mt)
        fd = os.open(os.devnull, os.O_WRONLY)
        try:
            t0 = time.perf_counter()
            c, nbytes, capped = refcpu.run_pairs_text(sq, qoff, sd, doff, m, fd,
                                                      max_pops=CPU_MAX_POPS, threads=T,
                                                      max_blocks=max_blocks)
            dt = time.perf_counter() - t0
        finally:
            os.close(fd)
        t0 = time.perf_counter()
        c2, capped2 = refcpu.run_pairs_capped(sq, qoff, sd, doff, m, max_pops=CPU_MAX_POPS,
                                              threads=T, max_blocks=max_blocks)
        dt2 = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": round(c / dt / 1e9, 5), "unit": "GCUPS", "cores": T,
                               "kind": "port", "capped_pairs": int(capped),
                               "text_bytes": int(nbytes), "seconds": round(dt, 3),
                               "sample": f"all {m} pairs of the file, oracle/refcpu.c fill + "
                                         f"literal DFS {blk} (<= {CPU_MAX_POPS:.0e} pops) on "
                                         f"{T} threads, each pair's reference text formatted "
                                         f"and written to /dev/null in pair order "
                                         f"(refmt.c), {dt:.2f} s; in-process (no process "
                                         f"start, which the CLI's value includes)",
                               "no_text": {"value": round(c2 / dt2 / 1e9, 5),
                                           "seconds": round(dt2, 3),
                                           "capped_pairs": int(capped2),
                                           "note": "the same DFS without formatting or "
                                                   "writing any text"}}
        res["vs_cpu_baseline"] = round(res["value"] / res["cpu_baseline"]["value"], 2)
    return res


C4_SHARDED_TIMEOUT_S = 180.0


def _leg_watchdog(rank, out, extra, leg, seconds):
    """A timer that, if `leg` has not finished after `seconds`, prints rank
    0's line (the headline and the legs so far, this one marked as timed out)
    and ends every rank's process (os._exit: no exec, no collective)."""
    import threading

    def fire():
        if rank == 0 and out is not None:
            o = dict(out)
            o["configs"] = dict(extra, **{leg: {"error": f"timed out after {seconds:.0f} s"}})
            print(json.dumps(o), flush=True)
        sys.stderr.flush()
        os._exit(0)

    t = threading.Timer(seconds, fire)
    t.daemon = True
    t.start()
    return t


# --------------------------------------------------------------- launcher
def launch_ranks(n: int) -> int:
    """Start n ranks of this command (torch.distributed.run, one process per
    GPU, rendezvous on 127.0.0.1) as a child and return its exit status.
    The parent never initialises the GPU (it must not, before a child that
    will use it starts)."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr", "127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    log(f"[bench] launching {n} ranks: torch.distributed.run --nproc-per-node={n} ...")
    return subprocess.call(cmd, env=env)


def launch_selftest(backend: str) -> None:
    """--selftest-launch: the ranks meet, agree on the world and print one
    JSON line (rank 0); no GPU work.  tests/test_bench_launch.py runs it on
    gloo."""
    import torch
    import torch.distributed as dist
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    diag = None
    if world > 1:
        dist.init_process_group(backend)
        t = torch.tensor([rank], dtype=torch.int64)
        ranks = [torch.zeros_like(t) for _ in range(world)]
        dist.all_gather(ranks, t)
        ranks = sorted(int(x.item()) for x in ranks)
        # the multi-GPU diagnosis of the real lines on a host stand-in: a
        # per-rank "compute" step and the gather of its records to rank 0
        rec = torch.full((4096,), rank, dtype=torch.int32)
        parts = [torch.empty_like(rec) for _ in range(world)] if rank == 0 else None
        t0 = time.perf_counter()
        _ = np.sort(np.random.default_rng(rank).random(200_000))
        compute_s = time.perf_counter() - t0
        gather_s = gather_probe(dist, torch, world, lambda: dist.gather(rec, parts, dst=0), 2)
        diag = rank_diag(dist, torch, world, "cpu", compute_s, gather_s,
                         rec.numel() * 4 * (world if rank == 0 else 1))
        dist.destroy_process_group()
    else:
        ranks = [0]
    if rank == 0:
        print(json.dumps({"launch_selftest": True, "n_gpus": world, "ranks": ranks,
                          "rank_diag": diag}), flush=True)


def main() -> None:
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--pairs", type=int, default=N_PAIRS)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--legs", default="auto",
                    help="comma list of extra configs (c2_full,c5,c1,c3,c3_affine,c4,c4_spans,host,"
                         "cli,cli_all; c4_sharded at N > 1), 'none', or 'auto' (all at N = 1, "
                         "c5 and c4_sharded at N > 1)")
    ap.add_argument("--score-only", action="store_true",
                    help="score + panic status only (no parent codes / traceback; the C5 mode)")
    ap.add_argument("--no-pipeline", dest="pipeline", action="store_false",
                    help="sequential steps: each step's traceback before the next step's fill "
                         "(default: step k's traceback on the engine's second stream beside "
                         "step k+1's fill; 2,298-2,337 vs 2,168-2,185 GCUPS on one box, r04)")
    ap.add_argument("--selftest-launch", action="store_true",
                    help="only start the ranks and report the world (no GPU work; tests)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend (nccl = RCCL)")
    args = ap.parse_args()
    bad = refused_env()
    if bad:
        sys.exit(f"bench.py: {', '.join(bad)} set in the environment; the bench measures the "
                 f"product library sequencealigning_amd/libsaln.so with its default options "
                 f"(allowed SALN_* variables: {', '.join(ALLOWED_ENV) or 'none'})")
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None and args.gpus > 1:
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        sys.exit(f"bench.py: WORLD_SIZE={env_world} but --gpus {args.gpus}")
    if args.selftest_launch:
        launch_selftest(args.backend)
        return

    import torch
    import torch.distributed as dist

    import sequencealigning_amd as saln
    from sequencealigning_amd import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    if world > 1:
        dist.init_process_group(args.backend, device_id=torch.device("cuda", local))
    if args.legs == "auto":
        legs = list(ALL_LEGS) if world == 1 else ["c5", "c4_sharded"]
    elif args.legs == "none":
        legs = []
    else:
        legs = [x for x in args.legs.split(",") if x]

    n = args.pairs
    qs, qo, ds, do = synth.iid_pairs(n, LQ, LD, seed=SEED + rank)
    plan = saln.NwPlan(qo, do, pairs=np.stack([np.arange(n), np.arange(n)], 1), device=local)
    dq = torch.from_numpy(qs).to(f"cuda:{local}")
    dd = torch.from_numpy(ds).to(f"cuda:{local}")
    # pipelined (default): the traceback of step k runs on the engine's second
    # stream while step k+1 fills; results/cigar/mask are double-buffered and
    # every step's results are complete (and gathered) inside the timed region.
    pipelined = args.pipeline and not args.score_only
    plan.set_score_only(args.score_only)
    plan.set_async(pipelined)
    nbuf = 2 if pipelined else 1
    res = [torch.zeros(n * 4, dtype=torch.int32, device=f"cuda:{local}") for _ in range(nbuf)]
    cig = [torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device=f"cuda:{local}")
           for _ in range(nbuf)]
    gathered = ([torch.empty_like(res[0]) for _ in range(world)] if (world > 1 and rank == 0)
                else None)
    state = {"k": 0}

    def gather(buf):
        if world > 1:
            dist.gather(res[buf], gathered, dst=0)

    def step():
        k = state["k"]
        buf = k % nbuf
        plan.execute(dq, dd, res[buf], cig[buf])
        state["k"] = k + 1
        if pipelined:
            if k > 0 and world > 1:
                plan.sync(keep_latest=True)  # results of step k-1 are complete
                gather((k - 1) % nbuf)
        else:
            gather(buf)

    def drain():
        if pipelined:
            plan.sync()
            if state["k"] > 0:
                gather((state["k"] - 1) % nbuf)
        state["k"] = 0

    for _ in range(args.warmup):
        step()
    drain()
    torch.cuda.synchronize()
    plan.set_timing(True)

    def run_steps():
        for _ in range(args.steps):
            step()
        drain()
    dt = timed(run_steps, world, dist, torch, local)
    local_dt = timed.local_s
    plan.check()  # device-side status of every timed execute (raises on a timeout)
    fill_ms, fill_n = plan.kernel_time("nw_fill")
    tb_ms, tb_n = plan.kernel_time("nw_traceback")
    ex_ms, ex_n = plan.kernel_time("nw_execute")
    diag = None
    if world > 1:
        # where a rank's step time went: its executes (events, per step) and
        # one RCCL gather of its records (probed after the timed region)
        g_s = gather_probe(dist, torch, world, lambda: gather(0))
        diag = rank_diag(dist, torch, world, f"cuda:{local}", ex_ms / max(1, ex_n) / 1e3, g_s,
                         res[0].numel() * 4 * (world if rank == 0 else 1),
                         wall_s=local_dt / max(1, args.steps))
    cells_rank = plan.cells
    total_cells = cells_rank * world * args.steps
    # outside the timed region: the fill alone (sequential executes), so the
    # line carries the kernel's own duration beside its co-run one
    fill_alone_s = None
    if pipelined and rank == 0:
        plan.set_async(False)
        plan.set_timing(True)
        for _ in range(5):
            plan.execute(dq, dd, res[0], cig[0])
        torch.cuda.synchronize(local)
        plan.check()
        fa_ms, fa_n = plan.kernel_time("nw_fill")
        fill_alone_s = fa_ms / max(1, fa_n) / 1e3
    gcups = total_cells / dt / 1e9
    fill_avg_s = fill_ms / max(1, fill_n) / 1e3
    out = None
    if rank == 0:
        last = (args.steps - 1) % nbuf if args.steps else 0
        hr = res[last].cpu().numpy()
        statuses = np.bincount(hr[1::4] & 0xFF, minlength=3)
        # 8 x 19 groups, 4-bit walk codes (table penalties unless nw.pk_tab = 0)
        fill_kernel = ("nw_fill_pk_tab_kernel<8, 19," if saln._lib.get_option("nw.pk_tab")[0]
                       else "nw_fill_pk_kernel<8, 19, 3,")
        roof = roof_hbm(cells_rank, fill_avg_s, "nw_fill",
                        pmc(fill_kernel) if not args.score_only else None,
                        traffic_unit="bytes/launch (PMC FETCH_SIZE*2 + WRITE_SIZE)",
                        traffic_source="profiles/pmc_traffic.json: rocprofv3 --pmc passes of "
                                       "this command (tools/pmc.sh), not measured in this run",
                        traceback_avg_ms=round(tb_ms / max(1, tb_n), 4),
                        execute_avg_ms=round(ex_ms / max(1, ex_n), 4), pipelined=pipelined,
                        step_frac=round(cells_rank / (dt / args.steps) / 1e9 / HBM_PEAK_GBS, 4),
                        kernel_avg_ms_alone=(round(fill_alone_s * 1e3, 4) if fill_alone_s
                                             else None),
                        frac_alone=(round(cells_rank / fill_alone_s / 1e9 / HBM_PEAK_GBS, 4)
                                    if fill_alone_s else None),
                        note=("pipelined: each fill co-runs with the previous step's traceback, "
                              "so kernel_avg_ms is the fill's co-run duration; "
                              "kernel_avg_ms_alone / frac_alone: 5 sequential executes after "
                              "the timed region; step_frac = algorithmic bytes per step / "
                              "ms_per_step / peak; algorithmic bytes = 1 B/cell (the parent "
                              "set, SURVEY 8(d)): the fill stores 4-bit walk codes, so its "
                              "written bytes (traffic) are below it") if pipelined else None,
                        valu=valu_roof(fill_kernel, fill_avg_s) if not args.score_only else None)
        roof["frac"] = round(roof["frac"], 4)
        out = {
            "metric": METRIC, "value": round(gcups, 3), "unit": "GCUPS", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": round(dt / args.steps * 1e3, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None,
            "dtype": "i32-exact (i16x2 packed arithmetic)",
            "data": "synthetic (splitmix64 G-iid ACGT)",
            "config": {"workload": ("configs[1]: independent 150x150 NW-affine pairs per GPU "
                                    "(fill storing 4-bit walk codes (0.5 B/cell: argI, argD, "
                                    "I-open, D-open) + first-printed traceback/CIGAR; the full "
                                    "1 B/cell parent-set variant is leg c2_full)")
                       if not args.score_only else
                       ("score-only 150x150 NW-affine pairs per GPU (the configs[4] per-pair "
                        "mode: score + panic status, no mask)"),
                       "pairs_per_gpu": n, "len_q": LQ, "len_db": LD, "seed": hex(SEED),
                       "parallelism": f"db-sharded x{world}" + (" + RCCL gather" if world > 1
                                                               else "")},
            "roofline": roof,
            "status_counts": {"ok": int(statuses[0]), "ref_panic_boundary": int(statuses[2])},
            "env": {k: os.environ[k] for k in ALLOWED_ENV if k in os.environ},
            "options": saln._lib.non_default_options(),
        }
        if diag is not None:
            out["rank_diag"] = {"per_step": diag,
                                "note": "compute_ms: the rank's execute (fill + walk) per step "
                                        "from hipEvents; gather_ms: one dist.gather of its "
                                        "records to rank 0 (RCCL), probed after the timed "
                                        "region; wall_ms: the rank's own timed wall per step"}
        if not args.score_only:
            out["verified"] = verify_c2(hr, cig[last].cpu().numpy().view(np.uint32),
                                        plan.cigar_off, qs, qo, ds, do)
    plan.close()
    del res, cig, dq, dd
    torch.cuda.empty_cache()

    cpu = not args.no_cpu_baseline
    extra = {}
    for leg in legs:
        t0 = time.perf_counter()
        try:
            if leg == "c5":
                r = leg_c5(world, rank, local, dist, torch, cpu=cpu)
            elif leg == "c4_sharded":
                if world < 2:
                    continue  # one span per rank: a multi-GPU leg
                # never run on >= 2 real RCCL ranks before: a watchdog ends a
                # stuck leg with the headline line still printed by rank 0
                wd = _leg_watchdog(rank, out, extra, leg, C4_SHARDED_TIMEOUT_S)
                try:
                    r = leg_c4_sharded(world, rank, local, dist, torch)
                except Exception as e:  # the line must survive this leg
                    r = {"error": f"{type(e).__name__}: {e}"}
                finally:
                    wd.cancel()
            elif rank != 0 or world > 1:
                continue
            elif leg == "c2_full":
                r = leg_c2_full(torch, saln)
            elif leg == "c1":
                r = leg_c1(torch, saln, cpu=cpu)
            elif leg == "c3":
                r = leg_c3(torch, saln, cpu=cpu)
            elif leg == "c3_affine":
                r = leg_c3_affine(torch, saln, cpu=cpu)
            elif leg == "c4":
                r = leg_c4(torch, saln, cpu=cpu)
            elif leg == "c4_spans":
                r = leg_c4_spans(torch, saln)
            elif leg == "host":
                r = leg_host(saln)
            elif leg == "cli":
                r = leg_cli(saln, cpu=cpu)
            elif leg == "cli_all":
                r = leg_cli(saln, n=316, cpu=cpu, max_blocks=0, gmut=True)
            else:
                raise ValueError(f"unknown leg {leg}")
        except Exception as e:  # a failing extra leg must not hide the headline line
            if world > 1:
                raise
            r = {"error": f"{type(e).__name__}: {e}"}
        if rank == 0:
            r["leg_wall_s"] = round(time.perf_counter() - t0, 2)
            extra[leg] = r
            log(f"[bench] {leg}: {json.dumps(r)[:300]}")
    _C3_PAIRS.clear()
    if rank == 0:
        if extra:
            out["configs"] = extra
        if cpu and world == 1:  # the CPU leg: rank 0 at N = 1 only
            out["cpu_baseline"] = cpu_baseline()
        print(json.dumps(out), flush=True)
    if world > 1:
        # the line is out: a teardown stuck behind a peer that left a leg
        # early (c4_sharded's error path) must not hold the job
        import threading
        t = threading.Timer(60.0, lambda: (sys.stderr.flush(), os._exit(0)))
        t.daemon = True
        t.start()
        dist.destroy_process_group()
        t.cancel()


if __name__ == "__main__":
    main()
