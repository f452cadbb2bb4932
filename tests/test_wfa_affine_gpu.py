"""GPU: the corrected gap-affine WFA engine (wfa_affine_kernels.hip,
SURVEY.md §8(f) row 4) returns the Gotoh DP's minimum penalty
(oracle/refaffine.c) on random, mutated, repetitive, empty and lopsided
pairs, through the host batch and the device-resident plan.  Not a
reference-parity path: the reference's wfa_align defines no output here
(SURVEY.md §8.5); `parity unpinned` against the reference."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _pairs(seed):
    from sequencealigning_amd import synth
    rng = np.random.default_rng(seed)
    qs, ds = [], []
    for k in range(96):
        kind = k % 6
        lq = int(rng.integers(1, 400))
        if kind == 0:   # i.i.d.
            q = synth.random_bases(seed * 1000 + k, lq).tobytes()
            d = synth.random_bases(seed * 1000 + k + 500, int(rng.integers(1, 400))).tobytes()
        elif kind == 1:  # mutated 5 %
            q = synth.random_bases(seed * 1000 + k, lq).tobytes()
            d = synth.mutate(q, 0.05, seed=k)
        elif kind == 2:  # mutated 20 %
            q = synth.random_bases(seed * 1000 + k, lq).tobytes()
            d = synth.mutate(q, 0.2, seed=k)
        elif kind == 3:  # repetitive, 2 letters
            q = bytes(rng.choice([65, 67], lq).astype(np.uint8))
            d = bytes(rng.choice([65, 67], int(rng.integers(1, 400))).astype(np.uint8))
        elif kind == 4:  # identical / prefix
            q = synth.random_bases(seed * 1000 + k, lq).tobytes()
            d = q[: int(rng.integers(0, lq + 1))]
        else:           # lopsided, with N
            q = bytes(rng.choice(list(b"ACGTN"), int(rng.integers(1, 30))).astype(np.uint8))
            d = bytes(rng.choice(list(b"ACGTN"), int(rng.integers(100, 500))).astype(np.uint8))
        qs.append(q)
        ds.append(d)
    qs += [b"", b"A", b"", b"ACGT"]
    ds += [b"", b"", b"ACG", b"ACGT"]
    return qs, ds


@pytest.mark.parametrize("pen", [(4, 2, 6), (1, 3, 1), (5, 0, 2), (3, 5, 1)])
def test_wfa_affine_matches_dp(saln, oracle, pen):
    qs, ds = _pairs(7)
    got = saln.wfa_affine.wfa_affine_batch(qs, ds, [(k, k) for k in range(len(qs))], penalties=pen)
    want = [oracle.affine_penalty(q, d, *pen) for q, d in zip(qs, ds)]
    assert got.tolist() == want


def test_wfa_affine_long_mutated_pairs(saln, oracle):
    """10 kbp G-mut(5 %) pairs (configs[2] shape): the second pass (wider
    ring) included, the penalties equal the DP's."""
    from sequencealigning_amd import synth
    qs = [synth.random_bases(900 + k, 10_000).tobytes() for k in range(3)]
    ds = [synth.mutate(q, 0.05, seed=950 + k) for k, q in enumerate(qs)]
    qs.append(synth.random_bases(990, 3000).tobytes())      # i.i.d.: wide wavefronts
    ds.append(synth.random_bases(991, 2500).tobytes())
    got = saln.wfa_affine.wfa_affine_batch(qs, ds, [(k, k) for k in range(len(qs))])
    want = [oracle.affine_penalty(q, d) for q, d in zip(qs, ds)]
    for g, w in zip(got.tolist(), want):
        assert g == w or (g == -2 and w > 5000), (g, w)


def test_wfa_affine_all_vs_all_and_cap(saln, oracle):
    from sequencealigning_amd import synth
    qs = [synth.random_bases(10 + k, 50 + 13 * k).tobytes() for k in range(5)]
    ds = [synth.mutate(qs[k % 5], 0.1, seed=k) for k in range(4)]
    got = saln.wfa_affine.wfa_affine_batch(qs, ds)  # db outer, query inner
    want = [oracle.affine_penalty(q, d) for d in ds for q in qs]
    assert got.tolist() == want
    capped = saln.wfa_affine.wfa_affine_batch(qs, ds, max_score=60)
    assert capped.tolist() == [w if w <= 60 else -1 for w in want]


def test_wfa_affine_device_plan(saln, oracle):
    import torch
    from sequencealigning_amd import synth
    qs = [synth.random_bases(300 + k, 200 + k).tobytes() for k in range(64)]
    ds = [synth.mutate(q, 0.08, seed=k) for k, q in enumerate(qs)]
    q_seq, q_off = saln.pack_csr(qs)
    d_seq, d_off = saln.pack_csr(ds)
    plan = saln.wfa_affine.WfaAffinePlan(q_off, d_off, [(k, k) for k in range(64)])
    dq = torch.from_numpy(q_seq).cuda()
    dd = torch.from_numpy(d_seq).cuda()
    sc = torch.full((64,), -7, dtype=torch.int32, device="cuda")
    plan.execute(dq, dd, sc)
    torch.cuda.synchronize()
    want = [oracle.affine_penalty(q, d) for q, d in zip(qs, ds)]
    assert sc.cpu().tolist() == want
    plan.close()
