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
