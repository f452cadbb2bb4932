"""GPU parity: libsaln's HIP NW-affine path vs the CPU oracle (oracle/refcpu.c,
a restatement of src/needleman_wunsch_affine.rs).  Bit-exact on scores, end
states, panic status, every parent code of every cell, the first printed
alignment and the full reference text."""
import json
import os

import numpy as np
import pytest

from nw_check import expand, path_score, rand_seq

pytestmark = pytest.mark.gpu

GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _compare(saln, oracle, q: bytes, d: bytes, *, mask=True, text=True, max_pops=200_000):
    o = oracle.nw(q, d, literal_dfs=text, max_pops=max_pops)
    r = saln.n_w_align(saln.Record(q, b">q"), saln.Record(d, b">d"))
    tag = f"q={q[:40]!r}.. ({len(q)}) d={d[:40]!r}.. ({len(d)})"
    assert r.score == o.score, tag
    assert r.end_states == o.end_states, tag
    assert r.panics == o.panics, tag
    assert r.printed == (o.first_ops is not None), tag
    if o.first_ops is not None:
        assert expand(r.cigar) == o.first_ops, tag
    if mask:
        dm = saln.dense_mask(q, d)
        if not np.array_equal(dm, o.dense_mask):
            bad = np.argwhere(dm != o.dense_mask)[:5]
            raise AssertionError(f"{tag}: mask differs at {bad.tolist()} "
                                 f"gpu={[int(dm[tuple(b)]) for b in bad]} "
                                 f"ref={[int(o.dense_mask[tuple(b)]) for b in bad]}")
    if text and o.dfs_rc != 2:
        t, nb, st = saln.render(q, d)
        assert t == o.stdout, tag
        assert nb == o.dfs_blocks, tag
        assert (st == 2) == (o.dfs_rc == 1), tag
    return r, o


def test_hand_kats(saln, oracle):
    """SURVEY.md §8.4 N1-N6 (hand-traced from needleman_wunsch_affine.rs)."""
    with open(os.path.join(GOLDEN, "nw_kats.json")) as f:
        kats = json.load(f)["hand"]
    for k in kats:
        q, d = k["query"].encode(), k["db"].encode()
        r = saln.n_w_align(q, d)
        assert r.score == k["score"], k["id"]
        t, nb, st = saln.render(q, d)
        assert t == k["stdout"], k["id"]
        assert (st == 2) == k["panics"], k["id"]


def test_golden_vectors(saln):
    """Committed oracle-generated vectors (tests/golden/make_golden.py)."""
    with open(os.path.join(GOLDEN, "nw_random.json")) as f:
        vecs = json.load(f)["pairs"]
    res, cig = saln.nw_align_batch([v["query"].encode() for v in vecs],
                                   [v["db"].encode() for v in vecs],
                                   pairs=[(k, k) for k in range(len(vecs))])
    for k, v in enumerate(vecs):
        assert int(res["score"][k]) == v["score"], k
        assert int(res["end_states"][k]) == v["end_states"], k
        assert (int(res["status"][k]) == 2) == v["panics"], k
        ops = expand(cig[k]) if res["printed"][k] else None
        assert ops == v["first_ops"], k


@pytest.mark.parametrize("lq,ld", [(1, 1), (2, 3), (7, 5), (16, 16), (31, 40), (150, 150),
                                   (160, 150), (161, 20), (200, 180), (256, 100), (257, 64),
                                   (300, 300), (512, 90), (513, 70), (1000, 1000),
                                   (1024, 30), (1025, 40), (2100, 33), (40, 2000),
                                   (100, 2600), (300, 4200)])  # last two: i32 lanes
def test_random_shapes(saln, oracle, lq, ld):
    rng = np.random.default_rng(lq * 7919 + ld)
    for rep in range(3):
        q = rand_seq(rng, lq)
        d = rand_seq(rng, ld)
        _compare(saln, oracle, q, d, text=lq * ld <= 40_000)


def test_mutated_and_ties(saln, oracle):
    from sequencealigning_amd import synth
    rng = np.random.default_rng(5)
    cases = [(b"A" * 30, b"A" * 25), (b"AC" * 20, b"CA" * 19), (b"ACGTN" * 10, b"NNNNN" * 8),
             (b"GATTACA", b"GATTACA"), (b"TA", b"A"), (b"AAA", b"AA")]
    for k in range(10):
        q, d = synth.mut_pair(int(rng.integers(20, 400)), 0.05, 1000 + k)
        cases.append((q, d))
    for q, d in cases:
        _compare(saln, oracle, q, d, text=len(q) * len(d) < 40_000, max_pops=100_000)


def test_empty_and_N(saln, oracle):
    for q, d in [(b"", b""), (b"", b"A"), (b"A", b""), (b"", b"ACGT" * 50), (b"N", b"N"),
                 (b"NNNN", b"NANN")]:
        _compare(saln, oracle, q, d, mask=len(q) > 0 and len(d) > 0)


def test_not_implemented_modes(saln):
    for m in (saln.Mode.Local, saln.Mode.SemiGlobal):
        with pytest.raises(saln.AlignmentError, match="not implemented"):
            saln.n_w_align(b"AC", b"AC", False, m)


def test_batch_ragged_all_vs_all(saln, oracle):
    rng = np.random.default_rng(11)
    qs = [rand_seq(rng, int(n)) for n in [0, 1, 5, 150, 151, 300, 700, 1030]]
    ds = [rand_seq(rng, int(n)) for n in [0, 3, 150, 222, 999]]
    res, cig = saln.nw_align_batch(qs, ds)  # all-vs-all, db outer / query inner
    assert len(res) == len(qs) * len(ds)
    for di, d in enumerate(ds):
        for qi, q in enumerate(qs):
            k = di * len(qs) + qi
            o = oracle.nw(q, d, literal_dfs=False)
            assert int(res["score"][k]) == o.score, (qi, di)
            assert int(res["end_states"][k]) == o.end_states
            assert (int(res["status"][k]) == 2) == o.panics
            assert (expand(cig[k]) if res["printed"][k] else None) == o.first_ops


def test_c2_scale_properties(saln, oracle):
    """configs[1]: 100k G-iid 150x150 pairs through the device plan, every
    pair checked against the oracle (literal fill + memoised DFS on the host
    cores, oracle/refcheck.c): score, end states, panic status, printed or
    not, and the first printed alignment word for word; every CIGAR also
    re-scores to its score under the reference recurrences."""
    import torch
    from sequencealigning_amd import synth
    n, L = 100_000, 150
    qs, qo, ds, do = synth.iid_pairs(n, L, L, seed=0x5EED0002)
    plan = saln.NwPlan(qo, do, pairs=np.stack([np.arange(n), np.arange(n)], 1))
    dq = torch.from_numpy(qs).cuda()
    dd = torch.from_numpy(ds).cuda()
    res_t = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
    cig_t = torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
    plan.execute(dq, dd, res_t, cig_t)
    torch.cuda.synchronize()
    res = res_t.cpu().numpy().view(saln._lib.RESULT_DTYPE)
    cig = cig_t.cpu().numpy().view(np.uint32)
    assert (res["flags"] == 0).all()
    want = oracle.check_pairs(qs, qo, ds, do)
    assert np.array_equal(res["score"], want.score)
    assert np.array_equal(res["end_states"], want.end_states)
    assert np.array_equal(res["status"] == saln._lib.REF_PANIC_BOUNDARY, want.panics)
    assert np.array_equal(res["printed"].astype(bool), want.cig_len >= 0)
    ops = {7: "=", 8: "X", 1: "I", 2: "D"}
    qb, db = qs.tobytes(), ds.tobytes()
    for k in range(n):
        if not res["printed"][k]:
            continue
        o0 = int(plan.cigar_off[k])
        got = cig[o0:o0 + int(res["cigar_len"][k])]
        assert np.array_equal(got, want.cigar_words(k)), k
        if k % 97 == 0:
            c = [(int(w) >> 4, ops[int(w) & 15]) for w in got]
            s, ok = path_score(qb[k * L:(k + 1) * L], db[k * L:(k + 1) * L], c)
            assert ok and s == int(res["score"][k]), k
    plan.close()


@pytest.mark.parametrize("tab", [1, 2, 3, 0])
def test_walk_code_formats_match_oracle(saln, oracle, saln_opt, tab):
    """The 4-bit walk codes of the short-query packed fills (8 x 19 groups for
    queries of <= 152 columns, 16 x 10 up to 160) give the oracle's results
    through both fills: the table fill (nw.pk_tab = 1, the default) and the
    generic one (nw.pk_tab = 0).  20,000 configs[1] pairs (score, end
    states, panic, printed, CIGAR word for word) and a ragged batch: 1..160-
    column queries, dbs up to 1,200 rows (the rebasing int16 frame),
    identical and two-letter pairs."""
    import torch
    from sequencealigning_amd import synth
    saln_opt("nw.pk_tab", tab)
    n, L = 20_000, 150
    qs, qo, ds, do = synth.iid_pairs(n, L, L, seed=0x5EED0002)
    plan = saln.NwPlan(qo, do, pairs=np.stack([np.arange(n), np.arange(n)], 1))
    dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
    res_t = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
    cig_t = torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
    plan.execute(dq, dd, res_t, cig_t)
    torch.cuda.synchronize()
    plan.check()
    res = res_t.cpu().numpy().view(saln._lib.RESULT_DTYPE)
    cig = cig_t.cpu().numpy().view(np.uint32)
    want = oracle.check_pairs(qs, qo, ds, do)
    assert np.array_equal(res["score"], want.score)
    assert np.array_equal(res["end_states"], want.end_states)
    assert np.array_equal(res["status"] == saln._lib.REF_PANIC_BOUNDARY, want.panics)
    assert np.array_equal(res["printed"].astype(bool), want.cig_len >= 0)
    for k in range(n):
        if res["printed"][k]:
            o0 = int(plan.cigar_off[k])
            assert np.array_equal(cig[o0:o0 + int(res["cigar_len"][k])], want.cigar_words(k)), k
    plan.close()
    rng = np.random.default_rng(4040 + 3 * tab)
    queries, dbs = [], []
    for lq, ld in [(1, 1), (1, 40), (9, 3), (19, 19), (20, 150), (38, 900), (151, 151),
                   (152, 152), (152, 1200), (153, 160), (160, 400), (140, 1200), (75, 5)]:
        queries.append(rand_seq(rng, lq))
        dbs.append(rand_seq(rng, ld))
    base = rand_seq(rng, 152)
    queries += [base, bytes(rng.choice([65, 67], 150).astype(np.uint8))]
    dbs += [base, bytes(rng.choice([65, 67], 147).astype(np.uint8))]
    m = len(queries)
    res, cg = saln.nw_align_batch(queries, dbs, pairs=[(k, k) for k in range(m)])
    for k in range(m):
        o = oracle.nw(queries[k], dbs[k], literal_dfs=False)
        assert (int(res["score"][k]), int(res["end_states"][k]), int(res["status"][k]) == 2) == \
            (o.score, o.end_states, o.panics), (k, len(queries[k]), len(dbs[k]))
        assert (saln.cigar_ops_string(cg[k]) if res["printed"][k] else None) == o.first_ops, k


def _run_plan(saln, qs, qo, ds, do, scoring=None):
    import torch
    n = len(qo) - 1
    plan = saln.NwPlan(qo, do, pairs=np.stack([np.arange(n), np.arange(n)], 1), scoring=scoring)
    dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
    res_t = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
    cig_t = torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
    plan.execute(dq, dd, res_t, cig_t)
    torch.cuda.synchronize()
    plan.check()
    res = res_t.cpu().numpy().view(saln._lib.RESULT_DTYPE).copy()
    cig = cig_t.cpu().numpy().view(np.uint32).copy()
    off = np.array(plan.cigar_off, copy=True)
    plan.close()
    return res, cig, off


@pytest.mark.parametrize("tab", [1, 2, 3])
@pytest.mark.parametrize("case", ["acgt", "with_n", "scheme", "long_db", "long_db_n"])
def test_table_fill_equals_generic(saln, oracle, saln_opt, case, tab):
    """nw.pk_tab = 1 (the 4-bit-code fill with table penalties in the
    extension-free frame, and its fallback launch for the waves whose pairs
    hold a byte other than A, C, G, T) equals nw.pk_tab = 0 on 20,000
    configs[1]-shaped pairs: every result field and every CIGAR word.  "acgt"
    is also checked against the oracle pair by pair; "with_n" puts an N into
    1 % of the queries and 1 % of the dbs (those waves take the fallback
    launch, the rest of the launch the table body); "scheme" uses
    {2, -3, -5, -2} (bonuses 12 / 2).  "long_db" / "long_db_n": 150 x 500
    pairs (8 x 19 groups) and 155 x 500 pairs (16 x 10
    groups), whose dbs need the rebasing frame in the original frame but not
    in the extension-free one (the fallback launch then rebases).  tab = 1:
    the scale-2 table body (the default), 2: scale 4 (round 6; values 4x + p,
    full-rate subtracts for the walk tests), 3: scale 2 with row profiles
    (round 6; one v_perm per column bonus, no xor)."""
    from sequencealigning_amd import synth
    n, L = 20_000, 150
    LD = L
    if case.startswith("long_db"):
        n, LD = 4_000, 500
    qs, qo, ds, do = synth.iid_pairs(n, L, LD, seed=0x7AB0 + len(case))
    if case.startswith("long_db"):  # the same db against a 155-column query (16 x 10)
        qs2, qo2, _, _ = synth.iid_pairs(n, 155, LD, seed=0x7AB1 + len(case))
        qs = np.concatenate([qs, qs2])
        qo = np.concatenate([qo, qo2[1:] + qo[-1]])
        ds = np.concatenate([ds, ds])
        do = np.concatenate([do, do[1:] + do[-1]])
        n *= 2
    qs, ds = qs.copy(), ds.copy()
    scoring = (2, -3, -5, -2) if case == "scheme" else None
    if case in ("with_n", "long_db_n"):
        rng = np.random.default_rng(77)
        for buf, off in ((qs, qo), (ds, do)):
            for k in rng.choice(n, n // 100, replace=False):
                buf[int(off[k]) + int(rng.integers(L))] = ord("N")
    saln_opt("nw.pk_tab", tab)
    r1, c1, o1 = _run_plan(saln, qs, qo, ds, do, scoring)
    saln_opt("nw.pk_tab", 0)
    r0, c0, o0 = _run_plan(saln, qs, qo, ds, do, scoring)
    assert np.array_equal(r1, r0)
    assert np.array_equal(o1, o0) and np.array_equal(c1, c0)
    if case in ("acgt", "long_db"):
        want = oracle.check_pairs(qs, qo, ds, do)
        assert np.array_equal(r1["score"], want.score)
        assert np.array_equal(r1["end_states"], want.end_states)
        assert np.array_equal(r1["status"] == saln._lib.REF_PANIC_BOUNDARY, want.panics)
        for k in range(0, n, 7):
            if r1["printed"][k]:
                got = c1[int(o1[k]):int(o1[k]) + int(r1["cigar_len"][k])]
                assert np.array_equal(got, want.cigar_words(k)), k


@pytest.mark.parametrize("lens", [(150, 150), (150, 156)])
def test_table_fill_concurrent_plans(saln, saln_opt, lens):
    """Two plans whose data hold N bytes execute at the same time on two
    streams, three times each: each plan's table launches mark their
    bail-outs in the plan's own bail word (a process-wide slot
    ring shared by the instantiations), so each fallback launch runs exactly
    its own launch's bail-outs.  (150, 156): the 8 x 19 table fill beside
    the 16 x 10 one.  Results equal each plan run alone."""
    import torch
    from sequencealigning_amd import synth
    saln_opt("nw.pk_tab", 1)
    n = 8_000
    data, plans, alone = [], [], []
    for seed, L in zip((0xC0, 0xC1), lens):
        qs, qo, ds, do = synth.iid_pairs(n, L, L, seed=seed)
        qs = qs.copy()
        rng = np.random.default_rng(seed)
        for k in rng.choice(n, n // 50, replace=False):
            qs[int(qo[k]) + int(rng.integers(L))] = ord("N")
        data.append((qs, qo, ds, do))
        alone.append(_run_plan(saln, qs, qo, ds, do))
    streams = [torch.cuda.Stream(), torch.cuda.Stream()]
    bufs = []
    for (qs, qo, ds, do) in data:
        plan = saln.NwPlan(qo, do, pairs=np.stack([np.arange(n), np.arange(n)], 1))
        dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
        res_t = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
        cig_t = torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
        plans.append(plan)
        bufs.append((dq, dd, res_t, cig_t))
    torch.cuda.synchronize()
    for _ in range(3):
        for plan, (dq, dd, res_t, cig_t), st in zip(plans, bufs, streams):
            plan.execute(dq, dd, res_t, cig_t, stream=st.cuda_stream)
    torch.cuda.synchronize()
    for plan, (dq, dd, res_t, cig_t), (r0, c0, _) in zip(plans, bufs, alone):
        plan.check()
        res = res_t.cpu().numpy().view(saln._lib.RESULT_DTYPE)
        assert np.array_equal(res, r0)
        assert np.array_equal(cig_t.cpu().numpy().view(np.uint32), c0)
        plan.close()


def test_pipelined_plan_matches_sync(saln):
    """saln_nw_plan_set_async: tracebacks overlap the next fill through two
    mask workspaces; five pipelined executes (ragged lengths, several
    variants, different inputs per step) must equal the synchronous plan byte
    for byte."""
    import torch
    from sequencealigning_amd import synth
    rng = np.random.default_rng(5)
    n = 3000
    lq = rng.integers(0, 400, n)
    ld = rng.integers(0, 400, n)
    lq[:5] = 0
    qo = np.zeros(n + 1, np.uint64); qo[1:] = np.cumsum(lq)
    do = np.zeros(n + 1, np.uint64); do[1:] = np.cumsum(ld)
    pairs = np.stack([np.arange(n), np.arange(n)], 1)
    sync_plan = saln.NwPlan(qo, do, pairs=pairs)
    pipe = saln.NwPlan(qo, do, pairs=pairs)
    pipe.set_async(True)
    steps = 5
    ins, want = [], []
    for s in range(steps):
        qs = synth.random_bases(100 + s, int(qo[-1]))
        ds = synth.random_bases(200 + s, int(do[-1]))
        dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
        r = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
        c = torch.zeros(max(1, sync_plan.cigar_words), dtype=torch.int32, device="cuda")
        sync_plan.execute(dq, dd, r, c)
        ins.append((dq, dd))
        want.append((r, c))
    got = []
    for s in range(steps):
        r = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
        c = torch.zeros(max(1, pipe.cigar_words), dtype=torch.int32, device="cuda")
        pipe.execute(*ins[s], r, c)
        got.append((r, c))
        pipe.sync(keep_latest=True)
    pipe.sync()
    torch.cuda.synchronize()
    for s in range(steps):
        assert torch.equal(got[s][0], want[s][0]), s
        assert torch.equal(got[s][1], want[s][1]), s
    sync_plan.close()
    pipe.close()


def test_score_only_plan_matches_full(saln):
    """saln_nw_plan_set_score_only (C5 mode): same scores and panic statuses
    as the full fill + traceback, over packed and i32 variants and empty sides."""
    import torch
    from sequencealigning_amd import synth
    rng = np.random.default_rng(8)
    n = 2000
    lq = rng.integers(0, 700, n)
    ld = rng.integers(0, 700, n)
    qo = np.zeros(n + 1, np.uint64); qo[1:] = np.cumsum(lq)
    do = np.zeros(n + 1, np.uint64); do[1:] = np.cumsum(ld)
    qs = torch.from_numpy(synth.random_bases(41, int(qo[-1]))).cuda()
    ds = torch.from_numpy(synth.random_bases(42, int(do[-1]))).cuda()
    pairs = np.stack([np.arange(n), np.arange(n)], 1)
    full = saln.NwPlan(qo, do, pairs=pairs)
    fast = saln.NwPlan(qo, do, pairs=pairs)
    fast.set_score_only(True)
    r1 = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
    r2 = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
    full.execute(qs, ds, r1, None)
    fast.execute(qs, ds, r2, None)
    torch.cuda.synchronize()
    a = r1.cpu().numpy().reshape(n, 4)
    b = r2.cpu().numpy().reshape(n, 4)
    assert np.array_equal(a[:, 0], b[:, 0])          # score
    assert np.array_equal(a[:, 1], b[:, 1])          # status
    assert ((b[:, 3] >> 16) & 0xFF == 8).all()       # flags: score-only
    full.close()
    fast.close()


def test_packed_rebase_shapes(saln, oracle):
    """Pairs past one int16 frame (db up to 2,528 rows for <= 256 query
    columns, 4,096 for <= 512) run through the packed fill with its rebasing
    frame: identical and embedded pairs (the largest in-frame excursions:
    the diagonal gains while column 0 drifts), random and two-letter pairs;
    scores, end states, panics, first alignment and the full parent mask
    equal the oracle's, alone and in one batch."""
    from sequencealigning_amd import synth
    rng = np.random.default_rng(777)
    cases = []
    base = synth.random_bases(900, 2600).tobytes()
    cases.append((base[:512], base[:512]))                      # identical 512 x 512
    cases.append((base[700:1212], base[:2000]))                 # embedded 512 in 2,000
    cases.append((base[300:450], base[:1248]))                  # embedded 150 in 1,248
    cases.append((base[1000:1150], base[:2528]))                # embedded 150 in 2,528
    cases.append((rand_seq(rng, 400), rand_seq(rng, 4000)))     # random 400 x 4,000
    cases.append((rand_seq(rng, 256), rand_seq(rng, 1200)))     # random 256 x 1,200
    cases.append((bytes(rng.choice([65, 67], 160).astype(np.uint8)),
                  bytes(rng.choice([65, 67], 1000).astype(np.uint8))))  # two-letter
    q, d = synth.mut_pair(600, 0.05, 4242)
    cases.append((q[:300], d[:650]))                            # mutated prefix pair
    for q, d in cases:
        _compare(saln, oracle, q, d, text=False)
    res, cig = saln.nw_align_batch([q for q, _ in cases] + [b"ACGT" * 30],
                                   [d for _, d in cases] + [b"ACGA" * 30],
                                   pairs=[(k, k) for k in range(len(cases) + 1)])
    for k, (q, d) in enumerate(cases + [(b"ACGT" * 30, b"ACGA" * 30)]):
        o = oracle.nw(q, d, literal_dfs=False)
        assert int(res["score"][k]) == o.score, k
        assert int(res["end_states"][k]) == o.end_states, k
        assert (int(res["status"][k]) == 2) == o.panics, k
        assert (saln.cigar_ops_string(cig[k]) if res["printed"][k] else None) == o.first_ops, k


def test_wide_packed_variant(saln, oracle):
    """Queries of 513-1,024 columns in 64-lane packed groups with the centred
    rebasing frame when a plan holds many of them, through the column stripes
    when it holds few (a short query against a db past the narrow variants'
    staged rows rides along on the i32 lanes).  All give the oracle's score,
    end states, panics and first alignment."""
    from sequencealigning_amd import synth
    rng = np.random.default_rng(888)
    base = synth.random_bases(901, 4200).tobytes()
    cases = [(base[:1024], base[:1024]),                                  # identical 1,024
             (base[1000:1800], base[:3000]),                              # embedded 800 in 3,000
             (rand_seq(rng, 700), rand_seq(rng, 650)),
             (bytes(rng.choice([65, 67], 600).astype(np.uint8)),
              bytes(rng.choice([65, 67], 620).astype(np.uint8))),
             (rand_seq(rng, 150), rand_seq(rng, 3000))]                   # long db, short query
    q, d = synth.mut_pair(1000, 0.05, 4343)
    cases.append((q, d))
    want = [oracle.nw(q, d, literal_dfs=False) for q, d in cases]
    for q, d in cases[2:4]:
        _compare(saln, oracle, q, d, text=False)                          # full parent mask
    reps = 1600 // 5 + 1   # five wide queries per round: > kWidePackedMinPairs, the packed variant
    for n in (1, reps):
        qs = [q for q, _ in cases] * n
        ds = [d for _, d in cases] * n
        res, cig = saln.nw_align_batch(qs, ds, pairs=[(k, k) for k in range(len(qs))])
        for k in range(len(qs)):
            o = want[k % len(cases)]
            assert int(res["score"][k]) == o.score, (n, k)
            assert int(res["end_states"][k]) == o.end_states, (n, k)
            assert (int(res["status"][k]) == 2) == o.panics, (n, k)
            if k < 2 * len(cases):
                assert (saln.cigar_ops_string(cig[k]) if res["printed"][k] else None) == o.first_ops, (n, k)


def test_packed_stripe_fill(saln, oracle, saln_opt):
    """The packed column-stripe fill, forced (option nw.stripe_pk = 1: int16 halves,
    128 virtual lanes, per-row frames) and its mask layout: stripe pairs alone
    (full parent mask, first alignment) and in a batch through the cooperative
    walker equal the oracle."""
    from sequencealigning_amd import synth
    saln_opt("nw.stripe_pk", 1)
    rng = np.random.default_rng(999)
    for lq, ld in [(513, 70), (1025, 40), (700, 900), (1300, 1280)]:
        _compare(saln, oracle, rand_seq(rng, lq), rand_seq(rng, ld), text=False)
    q, d = synth.mut_pair(2500, 0.05, 4545)
    cases = [(q, d), (rand_seq(rng, 1100), rand_seq(rng, 1000)),
             (bytes(rng.choice([65, 67], 1200).astype(np.uint8)),
              bytes(rng.choice([65, 67], 1150).astype(np.uint8)))]
    res, cig = saln.nw_align_batch([a for a, _ in cases], [b for _, b in cases],
                                   pairs=[(k, k) for k in range(len(cases))])
    for k, (a, b) in enumerate(cases):
        o = oracle.nw(a, b, literal_dfs=False)
        assert (int(res["score"][k]), int(res["end_states"][k]), int(res["status"][k]) == 2) == \
            (o.score, o.end_states, o.panics), k
        assert (saln.cigar_ops_string(cig[k]) if res["printed"][k] else None) == o.first_ops, k


def test_packed_stripes_auto_selected(saln, oracle, saln_opt):
    """A plan with >= 1,024 stripe waves (kStripePkMinWaves) of wide
    (>= 3,000-column) queries takes the packed stripe fill and layout by
    itself; a sample of its pairs equals the oracle, and every score equals
    the forced row-fill run's."""
    rng = np.random.default_rng(2024)
    n = 90  # 3,100-column queries: 13 chunks each, 1,170 waves
    qs = [rand_seq(rng, 3100) for _ in range(n)]
    ds = [rand_seq(rng, int(rng.integers(200, 320))) for _ in range(n)]
    pairs = [(k, k) for k in range(n)]
    res, cig = saln.nw_align_batch(qs, ds, pairs=pairs)
    for k in range(0, n, 9):
        o = oracle.nw(qs[k], ds[k], literal_dfs=False)
        assert (int(res["score"][k]), int(res["end_states"][k]), int(res["status"][k]) == 2) == \
            (o.score, o.end_states, o.panics), k
        assert (saln.cigar_ops_string(cig[k]) if res["printed"][k] else None) == o.first_ops, k
    saln_opt("nw.stripe_pk", 0)
    res0, cig0 = saln.nw_align_batch(qs, ds, pairs=pairs)
    assert res0["score"].tolist() == res["score"].tolist()
    assert res0["status"].tolist() == res["status"].tolist()
    assert all(saln.cigar_ops_string(a) == saln.cigar_ops_string(b) for a, b in zip(cig, cig0))


def test_context_block_cache_reuse(saln, oracle):
    """Plans of different sizes created and destroyed in turn on one context
    reuse its cached device blocks (dirty from the previous plan): results
    stay equal to the first run's and to the oracle's."""
    rng = np.random.default_rng(1212)
    batches = []
    for lq, ld, n in [(150, 150, 300), (1100, 900, 3), (40, 2000, 20), (700, 650, 4), (150, 150, 300)]:
        qs = [rand_seq(rng, lq) for _ in range(n)]
        ds = [rand_seq(rng, ld) for _ in range(n)]
        batches.append((qs, ds))
    first = []
    for qs, ds in batches:
        res, cig = saln.nw_align_batch(qs, ds, pairs=[(k, k) for k in range(len(qs))])
        first.append((res.copy(), cig))
    for rep in range(2):
        for (qs, ds), (r0, c0) in zip(batches[::-1], first[::-1]):
            res, cig = saln.nw_align_batch(qs, ds, pairs=[(k, k) for k in range(len(qs))])
            assert np.array_equal(res, r0) and cig == c0, rep
    for (qs, ds), (r0, c0) in zip(batches[1:4], first[1:4]):
        for k in range(min(3, len(qs))):
            o = oracle.nw(qs[k], ds[k], literal_dfs=False)
            assert (int(r0["score"][k]), int(r0["end_states"][k])) == (o.score, o.end_states)


@pytest.mark.parametrize("lq,ld", [(1, 5000), (5000, 1), (1025, 1), (1, 1025), (2, 3000),
                                   (600, 1), (513, 2), (1024, 1024), (1023, 3), (3, 4096)])
def test_degenerate_shapes_all_variants(saln, oracle, lq, ld):
    """Thin and boundary-sized pairs on every fill path (packed, rebasing,
    wide, i32 lanes, stripes), with N in the sequences: score, end states,
    panics, first alignment and the full parent mask equal the oracle's."""
    rng = np.random.default_rng(lq * 31 + ld)
    q = bytes(rng.choice(list(b"ACGTN"), lq).astype(np.uint8))
    d = bytes(rng.choice(list(b"ACGTN"), ld).astype(np.uint8))
    _compare(saln, oracle, q, d, text=False)


@pytest.mark.parametrize("L", [3000])
def test_long_pair_stripes(saln, oracle, L):
    """A single long mutated pair through the column-stripe fill (12 stripes of
    256 columns, pipelined): score, end states, status and the first printed
    alignment equal the oracle's."""
    from sequencealigning_amd import synth
    q = synth.random_bases(77, L).tobytes()
    d = synth.mutate(q, 0.05, seed=78)
    r = saln.n_w_align(q, d)
    o = oracle.nw(q, d, literal_dfs=False)
    assert r.score == o.score and r.end_states == o.end_states and r.panics == o.panics
    if o.first_ops is not None:
        assert expand(r.cigar) == o.first_ops


@pytest.mark.parametrize("shape", ["c4_mut_100k", "iid_20k", "wide_50k_x_3k", "tall_3k_x_50k",
                                   "narrow_400_x_60k"])
def test_very_long_pair_linear_oracle(saln, oracle, shape):
    """Pairs too large for the full-matrix oracle (configs[3] is 100 kbp x
    100 kbp): score, end states, panic status and the first printed alignment
    (or that nothing is printed) equal the linear-memory oracle's parent-set
    fill + literal DFS (oracle/reflinear.c), incl. pairs whose far corners
    are sentinel-rooted (narrow_400_x_60k prints nothing: every co-optimal
    path starts at a sentinel)."""
    from sequencealigning_amd import synth
    if shape == "c4_mut_100k":
        q = synth.random_bases(0x5EED0003, 100_000).tobytes()
        d = synth.mutate(q, 0.05, seed=100_000)
    elif shape == "iid_20k":
        q = synth.random_bases(21, 20_000).tobytes()
        d = synth.random_bases(22, 20_000).tobytes()
    else:
        lq, ld = {"wide_50k_x_3k": (50_000, 3_000), "tall_3k_x_50k": (3_000, 50_000),
                  "narrow_400_x_60k": (400, 60_000)}[shape]
        base = synth.random_bases(31, max(lq, ld)).tobytes()
        q = base[:lq]
        d = synth.mutate(base, 0.1, seed=32)[:ld]
    r = saln.n_w_align(q, d)
    sc, es, pan, first, _ = oracle.nw_first_linear(q, d)
    assert (r.score, r.end_states, r.panics) == (sc, es, pan)
    assert r.printed == (first is not None)
    if first is not None:
        assert expand(r.cigar) == first
        s, ok = path_score(q, d, r.cigar)
        assert ok and s == r.score


@pytest.mark.parametrize("passes", ["3", "1", "2"])
def test_speculative_stripe_walks_equal_sequential(saln, saln_opt, passes):
    """The speculative stripe walks of long column-stripe pairs (every
    256-column stripe walks at once, nw_traceback_coop_kernel kSpec) give the
    sequential walker's results exactly: accepted when linked (default 3
    passes), left to the cooperative walker when not (1 pass from guessed
    entries rarely links).  Single pairs and one plan of several."""
    from sequencealigning_amd import synth
    cases = []
    q = synth.random_bases(0x5EED0007, 30_000).tobytes()
    cases.append((q, synth.mutate(q, 0.05, seed=7)))
    q = synth.random_bases(0x5EED0008, 12_000).tobytes()
    cases.append((q, synth.mutate(q, 0.15, seed=8)))
    cases.append((synth.random_bases(41, 6_000).tobytes(), synth.random_bases(42, 6_500).tobytes()))
    base = synth.random_bases(43, 20_000).tobytes()
    cases.append((base, synth.mutate(base, 0.1, seed=44)[:2_500]))
    cases.append((base[:2_300], synth.mutate(base, 0.1, seed=45)))

    def run():
        single = [saln.n_w_align(q, d) for q, d in cases]
        res, cig = saln.nw_align_batch([c[0] for c in cases], [c[1] for c in cases],
                                       pairs=[(k, k) for k in range(len(cases))])
        return single, res, cig

    saln_opt("nw.spec", 0)
    seq = run()
    saln_opt("nw.spec", 1)
    saln_opt("nw.spec_passes", int(passes))
    spec = run()
    for a, b in zip(seq[0], spec[0]):
        assert (a.score, a.end_states, a.panics, a.printed) == (b.score, b.end_states, b.panics, b.printed)
        assert list(a.cigar) == list(b.cigar)
    assert np.array_equal(seq[1], spec[1])
    assert seq[2] == spec[2]


def test_speculative_stripe_walks_link(saln, saln_opt):
    """On mutated long pairs the three default passes link (option nw.spec_strict = 1
    turns a pair left to the cooperative walker into an error), so the
    speculative path, not the fallback, produced these results."""
    from sequencealigning_amd import synth
    saln_opt("nw.spec_strict", 1)
    q = synth.random_bases(0x5EED0009, 40_000).tobytes()
    d = synth.mutate(q, 0.05, seed=9)
    r = saln.n_w_align(q, d)
    s, ok = path_score(q, d, r.cigar)
    assert r.printed and ok and s == r.score


@pytest.mark.parametrize("k", ["1", "2"])
def test_row_fill_lane_widths_agree(saln, saln_opt, k):
    """The row fill's 64- and 128-column stripes (option nw.rows_k; a plan
    picks one itself) give identical results and CIGARs: a mutated
    12 kbp pair, a rectangular one and a batch of three."""
    from sequencealigning_amd import synth
    q = synth.random_bases(0x5EED000B, 12_000).tobytes()
    cases = [(q, synth.mutate(q, 0.05, seed=11)), (q[:7_000], synth.mutate(q, 0.1, seed=12)[:3_000])]
    saln_opt("nw.rows_k", 2)
    ref = [saln.n_w_align(a, b) for a, b in cases]
    ref_b = saln.nw_align_batch([c[0] for c in cases] + [q[:2_500]],
                                [c[1] for c in cases] + [q[100:2_700]],
                                pairs=[(0, 0), (1, 1), (2, 2)])
    saln_opt("nw.rows_k", int(k))
    got = [saln.n_w_align(a, b) for a, b in cases]
    got_b = saln.nw_align_batch([c[0] for c in cases] + [q[:2_500]],
                                [c[1] for c in cases] + [q[100:2_700]],
                                pairs=[(0, 0), (1, 1), (2, 2)])
    for x, y in zip(ref, got):
        assert (x.score, x.end_states, x.panics, x.printed) == (y.score, y.end_states, y.panics, y.printed)
        assert list(x.cigar) == list(y.cigar)
    assert np.array_equal(ref_b[0], got_b[0]) and ref_b[1] == got_b[1]


def test_deadend_pairs_device_plan(saln, oracle):
    """Pairs whose reference DFS leaves sentinel-rooted subtrees
    (tests/golden/nw_deadend.json, oracle-pinned): nothing printed, a panic
    found after a dead subtree, a block printed after one.  Through the
    single-pair path and one device plan holding all of them (i32 lanes and
    column stripes), every result equals the oracle's and no entry point
    reports an unresolved dead end."""
    with open(os.path.join(GOLDEN, "nw_deadend.json")) as f:
        pairs = json.load(f)["pairs"]
    qs = [p["query"].encode() for p in pairs]
    ds = [p["db"].encode() for p in pairs]
    for p, q, d in zip(pairs, qs, ds):
        r = saln.n_w_align(q, d)
        assert (r.score, r.end_states, r.panics) == (p["score"], p["end_states"], p["panics"]), p["id"]
        assert (expand(r.cigar) if r.printed else None) == p["first_ops"], p["id"]
    res, cig = saln.nw_align_batch(qs, ds, pairs=[(k, k) for k in range(len(qs))])
    assert (res["flags"] == 0).all()
    for k, p in enumerate(pairs):
        assert int(res["score"][k]) == p["score"] and int(res["end_states"][k]) == p["end_states"]
        assert (int(res["status"][k]) == 2) == p["panics"], p["id"]
        assert (expand(cig[k]) if res["printed"][k] else None) == p["first_ops"], p["id"]


@pytest.mark.parametrize("packed", [False, True])
def test_long_pairs_cooperative_walker(saln, oracle, packed):
    """Column-stripe pairs (> 512 query columns) take the cooperative
    traceback (one wave per pair, run-skipping over an LDS window of the
    mask): a batch of mutated, i.i.d. and tie-heavy long pairs, alone or
    sharing an interleaved mask pack, gives the oracle's score, end states,
    status and first printed alignment."""
    from sequencealigning_amd import synth
    rng = np.random.default_rng(4242)
    qs, ds = [], []
    shapes = [(1100, 1090), (1300, 1280), (1030, 1500), (1500, 700), (1025, 1030), (2000, 1900)]
    for k, (lq, ld) in enumerate(shapes):
        if k % 3 == 0:
            q = synth.random_bases(100 + k, lq).tobytes()
            d = synth.mutate(q, 0.05, seed=200 + k)[:ld]
        elif k % 3 == 1:
            q = synth.random_bases(100 + k, lq).tobytes()
            d = synth.random_bases(300 + k, ld).tobytes()
        else:  # two-letter alphabet: many co-optimal parents
            q = bytes(rng.choice([65, 67], lq).astype(np.uint8))
            d = bytes(rng.choice([65, 67], ld).astype(np.uint8))
        qs.append(q)
        ds.append(d)
    if packed:
        res, cig = saln.nw_align_batch(qs, ds, pairs=[(k, k) for k in range(len(qs))])
        got = [(int(res["score"][k]), int(res["end_states"][k]), int(res["status"][k]) == 2,
                saln.cigar_ops_string(cig[k]) if res["printed"][k] else None) for k in range(len(qs))]
    else:
        got = []
        for q, d in zip(qs, ds):
            r = saln.n_w_align(q, d)
            got.append((r.score, r.end_states, r.panics, expand(r.cigar) if r.printed else None))
    for k, (q, d) in enumerate(zip(qs, ds)):
        o = oracle.nw(q, d, literal_dfs=False)
        assert got[k][:3] == (o.score, o.end_states, o.panics), k
        assert got[k][3] == o.first_ops, k


def test_long_gaps_lds_walker(saln, oracle):
    """The LDS walker's I-run step (round 3: a run resolved from the lane's
    16-byte segment, at most nine cells per iteration, crossings into the
    previous block mid-run) and long D runs: pairs with gaps of 1-60 bases,
    at the ends too, through batches of packed variants 7 / 5 / 6 (10- and
    16-column blocks) and the i32 lanes, against the oracle's first printed
    alignment."""
    rng = np.random.default_rng(0x6A95)
    qs, ds = [], []
    for k in range(240):
        lq = int(rng.choice([150, 160, 240, 500]))
        base = rand_seq(rng, lq + 80)
        q = base[:lq]
        d = bytearray(q)
        for _ in range(int(rng.integers(1, 4))):
            at = int(rng.integers(0, len(d) + 1))
            g = int(rng.integers(1, 61))
            if rng.random() < 0.5 and len(d) > g + 1:  # deletion from the db: an I run
                del d[at:at + g]
            else:                                      # insertion into the db: a D run
                d[at:at] = rand_seq(rng, g)
        if k % 7 == 0:
            d = bytes(d)[:max(1, len(d) - int(rng.integers(1, 40)))]  # gap at the end
        qs.append(q)
        ds.append(bytes(d))
    res, cig = saln.nw_align_batch(qs, ds, pairs=[(k, k) for k in range(len(qs))])
    for k in range(len(qs)):
        o = oracle.nw(qs[k], ds[k], literal_dfs=False)
        assert int(res["score"][k]) == o.score, k
        assert int(res["end_states"][k]) == o.end_states, k
        assert (int(res["status"][k]) == 2) == o.panics, k
        assert (expand(cig[k]) if res["printed"][k] else None) == o.first_ops, k


def test_context_options_two_threads(saln, oracle):
    """Per-context options (saln_context_option_set): two
    contexts on two host threads run batches at the same time with
    different kernel choices - the 8 x 19 table fill (nw.pk_tab 1) and the
    generic 4-bit-code fill (pk_tab 0) - and both equal the oracle; the
    process registry and the per-process
    context keep their defaults."""
    import threading

    from sequencealigning_amd import _lib
    L = _lib.lib()
    rng = np.random.default_rng(91)
    n = 3_000
    qs = [rand_seq(rng, 150) for _ in range(n)]
    ds = [rand_seq(rng, int(rng.integers(120, 170))) for _ in range(n)]
    want = [oracle.nw(qs[k], ds[k], literal_dfs=False) for k in range(0, n, 10)]
    ctxs = [_lib.new_context(0), _lib.new_context(0)]
    try:
        default = _lib.get_option("nw.pk_tab")[1]
        _lib.set_context_option(ctxs[0], "nw.pk_tab", 1)
        _lib.set_context_option(ctxs[1], "nw.pk_tab", 0)
        assert _lib.get_context_option(ctxs[1], "nw.pk_tab") == 0
        assert _lib.get_option("nw.pk_tab")[0] == default
        assert _lib.get_context_option(_lib.context(0), "nw.pk_tab") == default
        out = [None, None]
        errs = []

        def run(i):
            try:
                rs = []
                for _ in range(3):  # overlapping repeats
                    rs.append(saln.nw_align_batch(qs, ds, pairs=[(k, k) for k in range(n)],
                                                  ctx=ctxs[i]))
                out[i] = rs
            except Exception as e:  # pragma: no cover - surfaced below
                errs.append(e)

        th = [threading.Thread(target=run, args=(i,)) for i in range(2)]
        for t in th:
            t.start()
        for t in th:
            t.join()
        assert not errs, errs
        for i in range(2):
            for res, cg in out[i]:
                for j, k in enumerate(range(0, n, 10)):
                    o = want[j]
                    assert (int(res["score"][k]), int(res["end_states"][k]),
                            int(res["status"][k]) == 2) == (o.score, o.end_states, o.panics), (i, k)
                    assert (saln.cigar_ops_string(cg[k]) if res["printed"][k] else None) == \
                        o.first_ops, (i, k)
        _lib.clear_context_option(ctxs[1])
        assert _lib.get_context_option(ctxs[1], "nw.pk_tab") == default
    finally:
        for c in ctxs:
            L.saln_context_destroy(c)


def test_pipelined_fallback_on_walk_stream(saln):
    """Pipelined plans queue the table fill's fallback launch (the waves whose
    pairs hold a byte other than A, C, G, T) on the walk stream behind the
    hand-off (round 5).  Steps alternate between inputs with ~1 % N bytes and
    clean ones, so a bailing step is followed by a fill into the other
    workspace while its fallback and walk run; each must equal the
    synchronous plan byte for byte."""
    import torch
    from sequencealigning_amd import synth
    n = 4000
    qs0, qo, ds0, do = synth.iid_pairs(n, 150, 150, seed=0x5EED0041)
    pairs = np.stack([np.arange(n)] * 2, 1)
    rng = np.random.default_rng(41)
    sync_plan = saln.NwPlan(qo, do, pairs=pairs)
    pipe = saln.NwPlan(qo, do, pairs=pairs)
    pipe.set_async(True)
    steps = 6
    ins, want = [], []
    for s in range(steps):
        qs, ds = qs0.copy(), ds0.copy()
        if s % 2 == 0:
            qs[rng.random(qs.size) < 0.01] = ord("N")
            ds[rng.random(ds.size) < 0.01] = ord("N")
        else:
            qs = np.roll(qs, s)
        dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
        r = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
        c = torch.zeros(max(1, sync_plan.cigar_words), dtype=torch.int32, device="cuda")
        sync_plan.execute(dq, dd, r, c)
        ins.append((dq, dd))
        want.append((r, c))
    got = []
    for s in range(steps):
        r = torch.full((n * 4,), -1, dtype=torch.int32, device="cuda")
        c = torch.zeros(max(1, pipe.cigar_words), dtype=torch.int32, device="cuda")
        pipe.execute(*ins[s], r, c)
        got.append((r, c))
    pipe.sync()
    pipe.check()
    torch.cuda.synchronize()
    for s in range(steps):
        assert torch.equal(got[s][0], want[s][0]), s
        assert torch.equal(got[s][1], want[s][1]), s
    sync_plan.close()
    pipe.close()


@pytest.mark.parametrize("waves", [-1, 1, 7])
def test_pipelined_mixed_variants_bail(saln, oracle, waves):
    """one async plan holding both 4-bit-code variants
    (150-column queries: 8 x 19; 156-column: 16 x 10) whose table fills both
    bail (N bytes in each), so both fallbacks are queued on the walk stream
    behind the two table launches.  Each variant has its own bail word; every
    step must equal the synchronous plan.  n = 4001 pairs (not a multiple of
    the walk grid's lanes) and explicit walk grids of 1 and 7 waves."""
    import torch
    from sequencealigning_amd import synth
    n = 4001
    lq = np.where(np.arange(n) % 2 == 0, 150, 156).astype(np.int64)
    ld = np.full(n, 150, np.int64)
    qo = np.concatenate([[0], np.cumsum(lq)]).astype(np.uint64)
    do = np.concatenate([[0], np.cumsum(ld)]).astype(np.uint64)
    qs0 = synth.random_bases(0x5EED0043, int(qo[-1]))
    ds0 = synth.random_bases(0x5EED0044, int(do[-1]))
    pairs = np.stack([np.arange(n)] * 2, 1)
    rng = np.random.default_rng(43)
    with saln.options(**{"nw.walk_waves": waves}):
        sync_plan = saln.NwPlan(qo, do, pairs=pairs)
        pipe = saln.NwPlan(qo, do, pairs=pairs)
    pipe.set_async(True)
    steps = 5
    ins, want = [], []
    for s in range(steps):
        qs, ds = qs0.copy(), ds0.copy()
        if s % 2 == 0:  # N bytes in pairs of both variants
            qs[rng.random(qs.size) < 0.004] = ord("N")
            ds[rng.random(ds.size) < 0.004] = ord("N")
        else:
            ds = np.roll(ds, s)
        dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
        r = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
        c = torch.zeros(max(1, sync_plan.cigar_words), dtype=torch.int32, device="cuda")
        sync_plan.execute(dq, dd, r, c)
        ins.append((dq, dd))
        want.append((r, c))
    got = []
    for s in range(steps):
        r = torch.full((n * 4,), -1, dtype=torch.int32, device="cuda")
        c = torch.zeros(max(1, pipe.cigar_words), dtype=torch.int32, device="cuda")
        pipe.execute(*ins[s], r, c)
        got.append((r, c))
    pipe.sync()
    pipe.check()
    sync_plan.check()
    torch.cuda.synchronize()
    for s in range(steps):
        assert torch.equal(got[s][0], want[s][0]), s
        assert torch.equal(got[s][1], want[s][1]), s
    # the N step against the oracle for every pair (both variants bailed)
    res = want[0][0].cpu().numpy().view(saln._lib.RESULT_DTYPE)
    cig = want[0][1].cpu().numpy().view(np.uint32)
    ref = oracle.check_pairs(ins[0][0].cpu().numpy(), qo, ins[0][1].cpu().numpy(), do)
    assert np.array_equal(res["score"], ref.score)
    assert np.array_equal(res["end_states"], ref.end_states)
    assert np.array_equal(res["printed"].astype(bool), ref.cig_len >= 0)
    for k in range(n):
        if res["printed"][k]:
            o0 = int(sync_plan.cigar_off[k])
            assert np.array_equal(cig[o0:o0 + int(res["cigar_len"][k])], ref.cigar_words(k)), k
    sync_plan.close()
    pipe.close()


@pytest.mark.parametrize("waves,length", [(1, 150), (6, 150), (48, 150)])
def test_walker_grid_in_turns(saln, waves, length):
    """nw.walk_waves caps the LDS walk launch of the 8 x 19 variant; each lane
    then walks several pairs in turn (round 5: two per lane beside the next
    fill by default).
    Sequential and pipelined plans with a capped grid equal the uncapped one."""
    import torch
    from sequencealigning_amd import synth
    n = 3000
    qs, qo, ds, do = synth.iid_pairs(n, length, length, seed=0x5EED0042)
    qs[::97] = ord("N")
    pairs = np.stack([np.arange(n)] * 2, 1)
    dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()

    def run(async_, opt):
        with saln.options(**{"nw.walk_waves": opt}):
            plan = saln.NwPlan(qo, do, pairs=pairs)
        plan.set_async(async_)
        out = []
        for _ in range(3):
            r = torch.full((n * 4,), -1, dtype=torch.int32, device="cuda")
            c = torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
            plan.execute(dq, dd, r, c)
            out.append((r, c))
        plan.sync()
        plan.check()
        torch.cuda.synchronize()
        plan.close()
        return out

    want = run(False, 0)
    for async_ in (False, True):
        for r, c in run(async_, waves):
            assert torch.equal(r, want[0][0]), (async_, waves)
            assert torch.equal(c, want[0][1]), (async_, waves)


@pytest.mark.parametrize("async_", [False, True])
def test_full_code_plan_c2(saln, oracle, async_):
    """The bench leg c2_full's path (saln_nw_plan_create_full): configs[1]
    pairs with the reference's full parent sets stored (1 B/cell), walked to
    the first printed CIGAR.  Every pair's score, end states, panic and CIGAR
    equal the oracle's (refcheck.c), and the parent sets read back from the
    plan (saln_nw_plan_dense_mask) equal the oracle's dense mask bit for bit
    on a sample, ragged shapes of every short-query variant included."""
    import torch
    from sequencealigning_amd import synth
    n, L = 20_000, 150
    qs, qo, ds, do = synth.iid_pairs(n, L, L, seed=0x5EED0002)
    pairs = np.stack([np.arange(n), np.arange(n)], 1)
    plan = saln.NwPlan(qo, do, pairs=pairs, full_codes=True)
    plan.set_async(async_)
    dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
    res_t = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
    cig_t = torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
    for _ in range(2):
        plan.execute(dq, dd, res_t, cig_t)
    plan.sync()
    plan.check()
    torch.cuda.synchronize()
    res = res_t.cpu().numpy().view(saln._lib.RESULT_DTYPE)
    cig = cig_t.cpu().numpy().view(np.uint32)
    want = oracle.check_pairs(qs, qo, ds, do)
    assert np.array_equal(res["score"], want.score)
    assert np.array_equal(res["end_states"], want.end_states)
    assert np.array_equal(res["status"] == saln._lib.REF_PANIC_BOUNDARY, want.panics)
    assert np.array_equal(res["printed"].astype(bool), want.cig_len >= 0)
    for k in range(n):
        if res["printed"][k]:
            o0 = int(plan.cigar_off[k])
            assert np.array_equal(cig[o0:o0 + int(res["cigar_len"][k])], want.cigar_words(k)), k
    if not async_:
        for k in range(0, n, 1999):
            q, d = qs[qo[k]:qo[k + 1]].tobytes(), ds[do[k]:do[k + 1]].tobytes()
            assert np.array_equal(plan.dense_mask(k), oracle.nw(q, d, literal_dfs=False).dense_mask), k
    plan.close()
    # ragged: every packed short/wide variant and the stripes in one full plan
    rng = np.random.default_rng(606)
    shapes = [(1, 1), (7, 300), (150, 150), (152, 40), (156, 156), (160, 900), (200, 200),
              (256, 1000), (300, 120), (512, 512), (700, 650), (1100, 300), (90, 2600)]
    qsl = [rand_seq(rng, a) for a, _ in shapes]
    dsl = [rand_seq(rng, b) for _, b in shapes]
    qcat, qo2 = saln.pack_csr(qsl)
    dcat, do2 = saln.pack_csr(dsl)
    m = len(shapes)
    plan = saln.NwPlan(qo2, do2, pairs=np.stack([np.arange(m)] * 2, 1), full_codes=True)
    r2 = torch.zeros(m * 4, dtype=torch.int32, device="cuda")
    c2 = torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
    plan.execute(torch.from_numpy(qcat).cuda(), torch.from_numpy(dcat).cuda(), r2, c2)
    plan.check()
    torch.cuda.synchronize()
    rr = r2.cpu().numpy().view(saln._lib.RESULT_DTYPE)
    for k in range(m):
        o = oracle.nw(qsl[k], dsl[k], literal_dfs=False)
        assert int(rr["score"][k]) == o.score, shapes[k]
        assert np.array_equal(plan.dense_mask(k), o.dense_mask), shapes[k]
    plan.close()


def test_full_code_table_fill_equals_generic(saln, oracle):
    """Round 6: full-code plans fill their 16-lane geometries (16 x 10 for
    queries of <= 160 columns, 16 x 16 for <= 256) with the table body and row
    profiles (nw.pk_tab != 0).  One async plan holds both variants; every
    other step puts N bytes into pairs of both, so both table launches bail
    and both fallbacks run behind them (a bail word per variant).  Every
    parent set of every pair equals the generic fill's (nw.pk_tab = 0) and, on
    a sample, the oracle's; results and CIGARs equal the synchronous generic
    plan's at every step."""
    import torch
    from sequencealigning_amd import synth
    n = 601
    lq = np.array([[150, 230, 157, 256, 1, 160][k % 6] for k in range(n)], np.int64)
    ld = np.array([[150, 300, 97, 150, 12, 1][k % 6] for k in range(n)], np.int64)
    qo = np.concatenate([[0], np.cumsum(lq)]).astype(np.uint64)
    do = np.concatenate([[0], np.cumsum(ld)]).astype(np.uint64)
    qs0 = synth.random_bases(0x5EED0061, int(qo[-1]))
    ds0 = synth.random_bases(0x5EED0062, int(do[-1]))
    pairs = np.stack([np.arange(n)] * 2, 1)
    with saln.options(**{"nw.pk_tab": 0}):
        gen = saln.NwPlan(qo, do, pairs=pairs, full_codes=True)
    tab = saln.NwPlan(qo, do, pairs=pairs, full_codes=True)
    tab.set_async(True)
    rng = np.random.default_rng(61)
    steps = 4
    ins, want, got = [], [], []
    for s_ in range(steps):
        qs, ds = qs0.copy(), ds0.copy()
        if s_ % 2 == 0:
            qs[rng.random(qs.size) < 0.003] = ord("N")
            ds[rng.random(ds.size) < 0.003] = ord("N")
        else:
            ds = np.roll(ds, s_)
        dq, dd = torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda()
        r = torch.zeros(n * 4, dtype=torch.int32, device="cuda")
        c = torch.zeros(max(1, gen.cigar_words), dtype=torch.int32, device="cuda")
        gen.execute(dq, dd, r, c)
        ins.append((dq, dd, qs, ds))
        want.append((r, c))
    for s_ in range(steps):
        r = torch.full((n * 4,), -1, dtype=torch.int32, device="cuda")
        c = torch.zeros(max(1, tab.cigar_words), dtype=torch.int32, device="cuda")
        tab.execute(ins[s_][0], ins[s_][1], r, c)
        got.append((r, c))
    tab.sync()
    tab.check()
    gen.check()
    torch.cuda.synchronize()
    for s_ in range(steps):
        assert torch.equal(got[s_][0], want[s_][0]), s_
        assert torch.equal(got[s_][1], want[s_][1]), s_
    # the last step's workspace: every parent set, table vs generic, and the
    # oracle's on a sample (N bytes included: step 2 bailed in both variants)
    last = steps - 2
    gen.execute(ins[last][0], ins[last][1], *want[last])
    tab.set_async(False)
    tab.execute(ins[last][0], ins[last][1], *got[last])
    torch.cuda.synchronize()
    qs, ds = ins[last][2], ins[last][3]
    for k in range(n):
        m = tab.dense_mask(k)
        assert np.array_equal(m, gen.dense_mask(k)), k
        if k % 37 == 0:
            q, d = qs[qo[k]:qo[k + 1]].tobytes(), ds[do[k]:do[k + 1]].tobytes()
            assert np.array_equal(m, oracle.nw(q, d, literal_dfs=False).dense_mask), k
    gen.close()
    tab.close()


@pytest.mark.parametrize("tab", [0, 1, 2, 3])
def test_walk_codes_bit_by_bit(saln, oracle, saln_opt, tab):
    """the 4-bit walk codes of the short-query fills
    (8 x 19 for <= 152 query columns, 16 x 10 up to 160), read back from the
    plan (saln_nw_plan_walk_codes), equal bit by bit what the reference's
    parent sets say for every cell the walker can read: argI / argD (I or D
    among the maxima at (i, j)), I-open (M + open among the maxima of I(i,
    j+1)), D-open (of D(i+1, j)), and argM at the end cell - through the
    generic fill (nw.pk_tab 0), the constant-table fill (1), scale 4 (2) and
    row profiles (3), with N bytes in some pairs (their waves take the
    fallback launch) and a db longer than the query's frame."""
    import torch
    saln_opt("nw.pk_tab", tab)
    rng = np.random.default_rng(707 + tab)
    shapes = [(150, 150)] * 6 + [(156, 156)] * 4 + [(152, 40), (140, 420), (160, 90), (37, 151)]
    qsl = [bytearray(rand_seq(rng, a)) for a, _ in shapes]
    dsl = [bytearray(rand_seq(rng, b)) for _, b in shapes]
    for k in (1, 7):  # N bytes: those waves go to the fallback launch
        qsl[k][int(rng.integers(len(qsl[k])))] = ord("N")
        dsl[k][int(rng.integers(len(dsl[k])))] = ord("N")
    base = rand_seq(rng, 150)  # tie-heavy: near-identical pair
    qsl.append(bytearray(base))
    dsl.append(bytearray(base[:70] + base[71:]))
    qsl, dsl = [bytes(x) for x in qsl], [bytes(x) for x in dsl]
    m = len(qsl)
    qcat, qo = saln.pack_csr(qsl)
    dcat, do = saln.pack_csr(dsl)
    plan = saln.NwPlan(qo, do, pairs=np.stack([np.arange(m)] * 2, 1))
    r = torch.zeros(m * 4, dtype=torch.int32, device="cuda")
    c = torch.zeros(max(1, plan.cigar_words), dtype=torch.int32, device="cuda")
    plan.execute(torch.from_numpy(qcat).cuda(), torch.from_numpy(dcat).cuda(), r, c)
    plan.check()
    torch.cuda.synchronize()
    for k in range(m):
        lq, ld = len(qsl[k]), len(dsl[k])
        got = plan.walk_codes(k)
        dm = oracle.nw(qsl[k], dsl[k], literal_dfs=False).dense_mask  # present bits
        inner = dm[1:, 1:]
        want_i = (inner & 2) == 0
        want_d = (inner & 4) == 0
        assert np.array_equal((got & 1) != 0, want_i), (k, "argI")
        assert np.array_equal((got & 2) != 0, want_d), (k, "argD")
        # I-open of I(i, j+1) at (i, j): columns 1 .. lq-1
        assert np.array_equal((got[:, :-1] & 4) != 0, (dm[1:, 2:] & 0x10) == 0), (k, "I-open")
        # D-open of D(i+1, j) at (i, j): rows 1 .. ld-1
        assert np.array_equal((got[:-1, :] & 8) != 0, (dm[2:, 1:] & 0x40) == 0), (k, "D-open")
        assert bool(got[ld - 1, lq - 1] & 8) == ((dm[ld, lq] & 1) == 0), (k, "argM")
    plan.close()
