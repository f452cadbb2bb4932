"""GPU: score-only all-vs-all (saln_nw_avsa_*, the configs[4] workload)
against the oracle — score and panic status of every (db, query) pair in the
reference order (src/main.rs:61-62: db outer, query inner)."""
import numpy as np
import pytest

from nw_check import rand_seq

pytestmark = pytest.mark.gpu


def test_avsa_mixed_lengths_vs_oracle(saln, oracle):
    rng = np.random.default_rng(5)
    q_lens = [0, 1, 7, 64, 149, 150, 151, 160, 161, 250, 300, 513, 700]
    d_lens = [0, 1, 5, 150, 151, 230, 399, 2]
    queries = [rand_seq(rng, n, b"ACGTN") for n in q_lens]
    dbs = [rand_seq(rng, n, b"ACGT") for n in d_lens]
    # a few near-identical pairs (long diagonals, ties)
    dbs.append(queries[5][:140] + b"AC")
    scores, status = saln.nw_score_all_vs_all(queries, dbs)
    assert scores.shape == (len(dbs), len(queries))
    for di, d in enumerate(dbs):
        for qi, q in enumerate(queries):
            o = oracle.nw(q, d, literal_dfs=False)
            assert scores[di, qi] == o.score, (qi, di)
            assert (status[di, qi] == saln._lib.REF_PANIC_BOUNDARY) == o.panics, (qi, di)


def test_avsa_matches_plan_at_scale(saln, oracle):
    """300 queries x 400 db records of ~150 bp (C5 shape): identical to the
    score-only plan over the explicit pair list, and a sample to the oracle."""
    import torch
    from sequencealigning_amd import synth
    rng = np.random.default_rng(9)
    nq, nd = 300, 400
    ql = rng.integers(120, 161, nq)
    dl = rng.integers(120, 161, nd)
    queries = [synth.random_bases(1000 + i, int(n)).tobytes() for i, n in enumerate(ql)]
    dbs = [synth.random_bases(5000 + i, int(n)).tobytes() for i, n in enumerate(dl)]
    scores, status = saln.nw_score_all_vs_all(queries, dbs)
    q_seq, q_off = saln.pack_csr(queries)
    d_seq, d_off = saln.pack_csr(dbs)
    plan = saln.NwPlan(q_off, d_off)          # all-vs-all pair list, reference order
    plan.set_score_only(True)
    res = torch.zeros(nq * nd * 4, dtype=torch.int32, device="cuda")
    plan.execute(torch.from_numpy(q_seq.copy()).cuda(), torch.from_numpy(d_seq.copy()).cuda(),
                 res, None)
    torch.cuda.synchronize()
    r = res.cpu().numpy().reshape(nd, nq, 4)
    plan.close()
    assert np.array_equal(r[..., 0], scores)
    assert np.array_equal(r[..., 1], status)
    for _ in range(40):
        di, qi = int(rng.integers(nd)), int(rng.integers(nq))
        o = oracle.nw(queries[qi], dbs[di], literal_dfs=False)
        assert scores[di, qi] == o.score


def test_avsa_full_configs4_sample(saln, oracle):
    """configs[4] at full size (10^4 x 10^5 pairs of 150 bp, 10^9 pairs, an
    8 GB result): a seeded sample of pairs spread over the whole index space
    equals the oracle (guards the launch chunking: a dispatch's grid is a
    32-bit work-item count)."""
    import torch
    from sequencealigning_amd import synth
    L, nq, ndb, seed = 150, 10_000, 100_000, 0x5EED0004
    qs = synth.random_bases(seed, nq * L)
    ds = synth.random_bases(seed ^ 0xD5D5D5D5, ndb * L)
    qo = np.arange(nq + 1, dtype=np.uint64) * np.uint64(L)
    do = np.arange(ndb + 1, dtype=np.uint64) * np.uint64(L)
    av = saln.NwAllVsAll(qo, do)
    out = torch.zeros(nq * ndb * 2, dtype=torch.int32, device="cuda")
    av.execute(torch.from_numpy(qs).cuda(), torch.from_numpy(ds).cuda(), out)
    torch.cuda.synchronize()
    rng = np.random.default_rng(7)
    di = np.concatenate([rng.integers(0, ndb, 200), [ndb - 1, ndb - 1, 0]])
    qi = np.concatenate([rng.integers(0, nq, 200), [nq - 1, 0, nq - 1]])
    pos = torch.from_numpy((di * nq * 2 + qi * 2).astype(np.int64)).cuda()
    sc = out[pos].cpu().numpy()
    st = out[pos + 1].cpu().numpy()
    allq, alld = qs.tobytes(), ds.tobytes()
    o2 = np.arange(len(di) + 1, dtype=np.uint64) * np.uint64(L)
    want = oracle.check_pairs(b"".join(allq[int(q) * L:(int(q) + 1) * L] for q in qi), o2,
                              b"".join(alld[int(d) * L:(int(d) + 1) * L] for d in di), o2)
    assert np.array_equal(sc, want.score)
    assert np.array_equal(st == saln._lib.REF_PANIC_BOUNDARY, want.panics)
    av.close()


def test_avsa_narrow_groups_equal_wide(saln, saln_opt):
    """Queries of <= 152 columns run in 8 x 19 lane groups (option nw.avsa_narrow,
    default on, dbs up to 600 rows); the 16 x 10 groups give the same score
    and status for every pair of a C5-shaped slice with ragged lengths and a
    db long enough to rebase the int16 frame."""
    rng = np.random.default_rng(11)
    queries = [rand_seq(rng, int(n)) for n in rng.integers(120, 153, 96)]
    dbs = [rand_seq(rng, int(n)) for n in rng.integers(100, 200, 60)] + [rand_seq(rng, 590)]
    saln_opt("nw.avsa_narrow", 1)
    a = saln.nw_score_all_vs_all(queries, dbs)
    saln_opt("nw.avsa_narrow", 0)
    b = saln.nw_score_all_vs_all(queries, dbs)
    assert np.array_equal(a[0], b[0]) and np.array_equal(a[1], b[1])


@pytest.mark.parametrize("nd,alphabet", [(401, b"ACGT"), (400, b"ACGT"), (201, b"ACGTN")])
def test_avsa_query_profiles_equal_generic(saln, saln_opt, oracle, nd, alphabet):
    """The 8 x 19 class with query profiles (nw.avsa_profile, AvsaSrcP: a
    group's two halves share the query; bonuses in the extension-free frame
    (nw.pk_tab = 1, the default) or penalties (nw.pk_tab = 0) from a
    per-column v_perm) equals the generic xor path on every pair: an odd db count (the last db
    record through AvsaSrc), and an N in the data (the device check selects
    the generic body inside the profile kernel).  A sample against the oracle."""
    rng = np.random.default_rng(nd)
    nq = 97
    queries = [rand_seq(rng, int(n), alphabet) for n in rng.integers(100, 153, nq)]
    dbs = [rand_seq(rng, int(n), alphabet) for n in rng.integers(100, 161, nd)]
    saln_opt("nw.avsa_profile", 1)
    s1, t1 = saln.nw_score_all_vs_all(queries, dbs)
    saln_opt("nw.pk_tab", 0)  # profiles of penalties in the original frame
    s2, t2 = saln.nw_score_all_vs_all(queries, dbs)
    saln_opt("nw.avsa_profile", 0)
    s0, t0 = saln.nw_score_all_vs_all(queries, dbs)
    assert np.array_equal(s1, s0) and np.array_equal(t1, t0)
    assert np.array_equal(s2, s0) and np.array_equal(t2, t0)
    for k in range(40):
        qi, di = int(rng.integers(nq)), int(rng.integers(nd))
        o = oracle.nw(queries[qi], dbs[di], literal_dfs=False)
        assert s1[di, qi] == o.score, (qi, di)
        assert (t1[di, qi] == saln._lib.REF_PANIC_BOUNDARY) == o.panics, (qi, di)


@pytest.mark.parametrize("lo,hi,alphabet", [(153, 256, b"ACGT"), (257, 512, b"ACGT"),
                                            (100, 600, b"ACGT"), (153, 256, b"ACGTN")])
def test_avsa_table_classes_equal_generic(saln, saln_opt, oracle, lo, hi, alphabet):
    """The query classes without profiles (16 x 16, 32 x 16, 16 x 10 / 8 x 19
    odd records) take table penalties in the extension-free frame under
    nw.pk_tab = 1 when every byte is A, C, G or T (the device check; with an
    N they keep the xor body): equal to nw.pk_tab = 0 on every pair, and a
    sample against the oracle."""
    rng = np.random.default_rng(lo * 7 + hi + len(alphabet))
    queries = [rand_seq(rng, int(n), alphabet) for n in rng.integers(lo, hi + 1, 61)]
    dbs = [rand_seq(rng, int(n), alphabet) for n in rng.integers(lo, hi + 1, 37)]
    saln_opt("nw.pk_tab", 1)
    s1, t1 = saln.nw_score_all_vs_all(queries, dbs)
    saln_opt("nw.pk_tab", 0)
    s0, t0 = saln.nw_score_all_vs_all(queries, dbs)
    assert np.array_equal(s1, s0) and np.array_equal(t1, t0)
    for _ in range(12):
        qi, di = int(rng.integers(len(queries))), int(rng.integers(len(dbs)))
        o = oracle.nw(queries[qi], dbs[di], literal_dfs=False)
        assert s1[di, qi] == o.score, (qi, di)
        assert (t1[di, qi] == saln._lib.REF_PANIC_BOUNDARY) == o.panics, (qi, di)
