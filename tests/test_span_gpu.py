"""GPU: one long pair split by query columns (SURVEY.md §8(f) #3,
saln_nw_span_* / sequencealigning_amd/span.py) against the oracle and the
single-GPU plan path (n_w_align), on the box's one GPU: the spans' fills run
concurrently and hand boundary rows over in bands (device copies behind
watch kernels), or one after another; 2-process gloo relay and 1-rank RCCL
runs of ShardedLongPair."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _mut(rng, q, rate):
    from nw_check import rand_seq
    out = bytearray()
    for c in q:
        u = rng.random()
        if u < rate / 2:
            out.append(ord("ACGT"[(int(rng.integers(1, 4)) + "ACGT".index(chr(c))) % 4]))
        elif u < 3 * rate / 4:
            out.append(c)
            out += rand_seq(rng, 1)
        elif u < rate:
            continue
        else:
            out.append(c)
    return bytes(out)


def _same(a, b):
    assert (a.score, a.status, a.end_states, a.printed) == (b.score, b.status, b.end_states,
                                                            b.printed)
    assert a.cigar == b.cigar


def _vs_oracle(r, qs, ds):
    from oracle import refcpu

    from sequencealigning_amd.nw import cigar_ops_string
    o = refcpu.nw(qs, ds, literal_dfs=False)
    assert r.score == o.score and (r.status == 2) == o.panics and r.end_states == o.end_states
    assert r.printed == (o.first_ops is not None)
    if r.printed:
        assert cigar_ops_string(r.cigar) == o.first_ops


@pytest.mark.parametrize("pipelined,cu_split", [(True, True), (True, False), (False, False)])
def test_span_chain_matches_oracle(pipelined, cu_split):
    """2-4 spans of mutated and iid pairs (up to 1.6 kbp): score, panic
    status, end states and first printed alignment equal the oracle's."""
    import sequencealigning_amd as saln
    from nw_check import rand_seq

    from sequencealigning_amd.span import nw_align_long_spans
    rng = np.random.default_rng(41)
    cases = []
    for lq, rate in [(1600, 0.05), (1100, 0.15), (800, 0.0)]:
        q = rand_seq(rng, lq)
        cases.append((q, _mut(rng, q, rate)))
    cases.append((rand_seq(rng, 900), rand_seq(rng, 1200)))  # iid, tall
    cases.append((rand_seq(rng, 1300), rand_seq(rng, 150)))  # iid, wide: end gaps, panics
    cases.append((b"ACGTN" * 120, b"AC" * 40))
    for qs, ds in cases:
        for n in (2, 3, 4):
            if (len(qs) + 255) // 256 < n:
                continue
            r = nw_align_long_spans(qs, ds, n, band_rows=128, pipelined=pipelined,
                                    cu_split=cu_split)
            _vs_oracle(r, qs, ds)
            _same(r, saln.n_w_align(qs, ds))


@pytest.mark.parametrize("spec", ["1", "0"])
def test_span_chain_long_pairs_match_plan(spec, saln_opt):
    """20-30 kbp pairs over 3-8 spans (pipelined, 2,048-row bands) give the
    single-GPU plan's result word for word, with the speculative span walks
    and with the sequential walker alone (option nw.spec = 0); a mask-free oracle
    pins the score."""
    saln_opt("nw.spec", int(spec))
    import sequencealigning_amd as saln
    from nw_check import rand_seq
    from oracle import refcpu

    from sequencealigning_amd.span import nw_align_long_spans
    rng = np.random.default_rng(42)
    for lq, ld_rate, n in [(30_000, 0.05, 8), (20_000, 0.10, 3)]:
        q = rand_seq(rng, lq)
        d = _mut(rng, q, ld_rate)
        r = nw_align_long_spans(q, d, n, band_rows=2048)
        _same(r, saln.n_w_align(q, d))
        sc, es, pan = refcpu.nw_score_linear(q, d)
        assert r.score == sc and r.end_states == es and (r.status == 2) == pan


def test_span_injected_timeout_raises():
    """A span whose inbox never arrives (no left neighbour ran) with a wait
    limit of 0 reports SALN_E_DEVICE_WAIT instead of hanging."""
    import torch

    from sequencealigning_amd import _lib
    from sequencealigning_amd.span import NwSpan
    q = torch.randint(65, 70, (1024,), dtype=torch.uint8, device="cuda")
    d = torch.randint(65, 70, (500,), dtype=torch.uint8, device="cuda")
    sp = NwSpan(1024, 500, 512, 1024, device=0)
    sp.set_wait_limit(0)
    sp.reset()
    sp.fill(q, d)
    with pytest.raises(_lib.SalnError, match="E_DEVICE_WAIT"):
        sp.check()
    sp.set_wait_limit(1 << 24)
    assert sp.status() == 0  # read and clear
    sp.close()


def test_span_relay_wait_limit_bounds_each_row():
    """The single-device relay (saln_nw_span_forward) under a small nonzero
    wait limit: its source rows arrive in 64-row batches ~5 ms apart for
    ~0.3 s, so the relay polls far longer in total than the limit allows one
    wait (2^17 polls: ~13-130 ms at 0.1-1 us a poll), but no single row waits
    long.  The limit bounds each row's wait: every row is
    forwarded, no timeout is flagged."""
    import time

    import torch

    from sequencealigning_amd import _lib
    from sequencealigning_amd.span import NwSpan
    R = 64 * 60
    a = NwSpan(512, R, 0, 256, device=0)
    b = NwSpan(512, R, 256, 512, device=0)
    a.reset()
    b.reset()
    torch.cuda.synchronize()
    a.set_wait_limit(1 << 17)
    vals = torch.arange(1, R + 1, dtype=torch.int64, device="cuda") * 3 + 7
    torch.cuda.synchronize()
    side = torch.cuda.Stream()
    _lib.check(_lib.lib().saln_nw_span_forward(a._h, b._h, 1, R, side.cuda_stream),
               "saln_nw_span_forward")
    # the writes go on a stream of their own (the null stream could wait for
    # the relay), and nothing here synchronizes the device before they are in
    writer = torch.cuda.Stream()
    t0 = time.perf_counter()
    with torch.cuda.stream(writer):
        for lo in range(1, R + 1, 64):
            time.sleep(0.005)
            a.outbox[lo:lo + 64].copy_(vals[lo - 1:lo + 63])
    side.synchronize()
    assert time.perf_counter() - t0 > 0.25  # the relay polled for the whole run
    torch.cuda.synchronize()
    assert a.status() == 0  # no wait gave up
    assert torch.equal(b.inbox[1:R + 1], vals)
    a.close()
    b.close()


def _relay_worker(rank, world, port, q, d, out):
    import torch
    import torch.distributed as dist

    from sequencealigning_amd.span import ShardedLongPair
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    sp = ShardedLongPair(q, d, device=0, band_rows=1000)
    r = sp.align()
    sp.close()
    if rank == 0:
        out.put((r.score, r.status, r.end_states, r.printed, r.cigar))
    dist.barrier()
    dist.destroy_process_group()


def test_sharded_long_pair_gloo_relay_gpu():
    """Two ranks (gloo; both on cuda:0) each fill one span of a 6 kbp pair on
    the GPU, boundary bands relayed through host memory: the result on rank 0
    equals the single-process plan's."""
    import sequencealigning_amd as saln
    from nw_check import rand_seq
    rng = np.random.default_rng(43)
    q = rand_seq(rng, 6000)
    d = _mut(rng, q, 0.08)
    ctx = mp.get_context("spawn")
    qu = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_relay_worker, args=(r, 2, port, q, d, qu)) for r in range(2)]
    for p in procs:
        p.start()
    got = qu.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    want = saln.n_w_align(q, d)
    assert got == (want.score, want.status, want.end_states, want.printed, want.cigar)


def _nccl_worker(port, q, d, out):
    import torch
    import torch.distributed as dist

    from sequencealigning_amd.span import ShardedLongPair
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    sp = ShardedLongPair(q, d, device=0)
    r = sp.align()
    sp.close()
    out.put((r.score, r.status, r.end_states, r.printed, r.cigar))
    dist.destroy_process_group()


def test_sharded_long_pair_rccl_single_rank():
    """ShardedLongPair's nccl (RCCL) path on one rank: the fill through the
    stream-ordered pipeline, the broadcasts and the gather of the run words
    over RCCL; equal to the plan path."""
    import sequencealigning_amd as saln
    from nw_check import rand_seq
    rng = np.random.default_rng(44)
    q = rand_seq(rng, 3000)
    d = _mut(rng, q, 0.05)
    ctx = mp.get_context("spawn")
    qu = ctx.Queue()
    p = ctx.Process(target=_nccl_worker, args=(_free_port(), q, d, qu))
    p.start()
    got = qu.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    want = saln.n_w_align(q, d)
    assert got == (want.score, want.status, want.end_states, want.printed, want.cigar)


@pytest.mark.parametrize("shape,n", [("c4_mut_100k", 8), ("iid_20k", 4), ("wide_50k_x_3k", 8),
                                     ("tall_3k_x_50k", 4)])
def test_span_chain_very_long_linear_oracle(shape, n):
    """configs[3]'s 100 kbp pair and other pairs too large for the full-matrix
    oracle, through n CU-partitioned spans: score, end states, panic status
    and the first printed alignment equal the linear-memory oracle's
    (oracle/reflinear.c parent-set fill + the reference DFS's first event),
    incl. an iid pair whose walks meet sentinel-rooted states."""
    from nw_check import path_score
    from oracle import refcpu

    from sequencealigning_amd import synth
    from sequencealigning_amd.nw import cigar_ops_string
    from sequencealigning_amd.span import nw_align_long_spans
    if shape == "c4_mut_100k":
        q = synth.random_bases(0x5EED0003, 100_000).tobytes()
        d = synth.mutate(q, 0.05, seed=100_000)
    elif shape == "iid_20k":
        q = synth.random_bases(21, 20_000).tobytes()
        d = synth.random_bases(22, 20_000).tobytes()
    else:
        lq, ld = {"wide_50k_x_3k": (50_000, 3_000), "tall_3k_x_50k": (3_000, 50_000)}[shape]
        base = synth.random_bases(31, max(lq, ld)).tobytes()
        q = base[:lq]
        d = synth.mutate(base, 0.1, seed=32)[:ld]
    r = nw_align_long_spans(q, d, n, band_rows=1024)
    sc, es, pan, first, _ = refcpu.nw_first_linear(q, d)
    assert (r.score, r.end_states, r.status == 2) == (sc, es, pan)
    assert r.printed == (first is not None)
    if first is not None:
        assert cigar_ops_string(r.cigar) == first
        s, ok = path_score(q, d, r.cigar)
        assert ok and s == r.score


@pytest.mark.parametrize("scoring", [(2, -3, -5, -2), (5, -4, -8, -20), (1, -1, -2, -1)])
def test_span_chain_custom_scoring_matches_plan(scoring):
    """Other scoring schemes through the spans equal the single-GPU plan's
    result word for word, incl. gap penalties large enough that the
    boundary row / column fall to the reference's -32768 sentinel inside a
    4 kbp pair (dead-end end states, nothing printed)."""
    import sequencealigning_amd as saln
    from nw_check import rand_seq

    from sequencealigning_amd.span import nw_align_long_spans
    rng = np.random.default_rng(45)
    q = rand_seq(rng, 4000)
    for d in (_mut(rng, q, 0.05), rand_seq(rng, 3500)):
        for n in (2, 5):
            r = nw_align_long_spans(q, d, n, scoring=scoring, band_rows=512)
            _same(r, saln.n_w_align(q, d, scoring=scoring))


def test_cu_range_streams_cover_every_xcd():
    """saln_stream_create_cu_range refuses a range that leaves an XCD without a
    mask bit (that XCD would run unmasked), and a range of 8k bits places its
    waves on k CUs of every XCD (bit c -> XCD c mod 8, profiles/r04_cu_map.json)."""
    import ctypes as C

    from sequencealigning_amd import _lib
    L, ctx = _lib.lib(), _lib.context(0)
    h = C.c_void_p()
    assert L.saln_stream_create_cu_range(ctx, 0, 4, C.byref(h)) == _lib.E_INVALID
    assert L.saln_stream_create_cu_range(ctx, 8, 24, C.byref(h)) == _lib.OK
    n = 256
    hw, xc = (C.c_uint32 * n)(), (C.c_uint32 * n)()
    try:
        assert L.saln_device_cu_probe(ctx, h, n, hw, xc) == _lib.OK
    finally:
        L.saln_stream_destroy(ctx, h)
    places = {(xc[k] & 0xF, (hw[k] >> 13) & 7, (hw[k] >> 12) & 1, (hw[k] >> 8) & 0xF) for k in range(n)}
    per_xcd = [sum(1 for p in places if p[0] == x) for x in range(8)]
    assert per_xcd == [2] * 8, per_xcd


def test_workgroup_dispatch_round_robin_over_xcds():
    """The row fill's XCD-local placement (nw_fill_rows_kernel kPlaceXcd)
    assumes workgroup b of a launch on an unmasked stream runs on XCD b % 8:
    wave v = (b % 8) * run + b / 8 then keeps runs of consecutive stripes on
    one XCD.  The probe records each one-wave workgroup's XCC_ID."""
    import ctypes as C

    from sequencealigning_amd import _lib
    L, ctx = _lib.lib(), _lib.context(0)
    n = 1024
    hw, xc = (C.c_uint32 * n)(), (C.c_uint32 * n)()
    assert L.saln_device_cu_probe(ctx, None, n, hw, xc) == _lib.OK
    ids = [xc[b] & 0xF for b in range(n)]
    assert len(set(ids[:8])) == 8, ids[:8]
    assert all(ids[b] == ids[b % 8] for b in range(n)), \
        [(b, ids[b], ids[b % 8]) for b in range(n) if ids[b] != ids[b % 8]][:8]


@pytest.mark.parametrize("lo,hi", [(0, 32), (96, 128), (0, 64)])
def test_workgroup_dispatch_round_robin_masked_stream(lo, hi):
    """On a CU-range stream (a span's 1/8 or 1/4 of the CUs, k CUs of every
    XCD) workgroup b still runs on XCD b % 8, so the row fill's XCD runs also
    hold for the spans' masked fills (xcd_fit)."""
    import ctypes as C

    from sequencealigning_amd import _lib
    L, ctx = _lib.lib(), _lib.context(0)
    st = C.c_void_p()
    assert L.saln_stream_create_cu_range(ctx, lo, hi, C.byref(st)) == _lib.OK
    try:
        n = 1024
        hw, xc = (C.c_uint32 * n)(), (C.c_uint32 * n)()
        assert L.saln_device_cu_probe(ctx, st, n, hw, xc) == _lib.OK
        ids = [xc[b] & 0xF for b in range(n)]
        assert len(set(ids[:8])) == 8, ids[:8]
        assert all(ids[b] == ids[b % 8] for b in range(n)), \
            [(b, ids[b], ids[b % 8]) for b in range(n) if ids[b] != ids[b % 8]][:8]
    finally:
        L.saln_stream_destroy(ctx, st)


@pytest.mark.parametrize("lq,ld", [(20000, 20000), (9000, 30000)])
def test_row_fill_xcd_placement_equal(saln_opt, lq, ld):
    """nw.rows_xcd = 1 (stripes in XCD runs, plain publication inside a run)
    gives the same scores, statuses and CIGARs as the dispatch-order placement."""
    from nw_check import rand_seq

    import sequencealigning_amd as saln
    rng = np.random.default_rng(lq + ld)
    q = rand_seq(rng, lq)
    d = _mut(rng, q, 0.05)[:ld] if ld <= lq else _mut(rng, q, 0.05) + rand_seq(rng, ld - lq)
    saln_opt("nw.rows_xcd", 0)
    a = saln.n_w_align(q, d)
    saln_opt("nw.rows_xcd", 1)
    b = saln.n_w_align(q, d)
    _same(a, b)
