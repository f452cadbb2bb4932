"""Seeded fuzz over mixed shapes in one plan (every fill variant side by side:
packed, rebasing, i32 lanes, column stripes, empty sides) against the CPU
oracle: score, end states, panic status and the first printed alignment."""
import numpy as np
import pytest

from nw_check import rand_seq


def _pairs(seed, n):
    from sequencealigning_amd import synth
    rng = np.random.default_rng(seed)
    out = []
    for k in range(n):
        lq = int(np.exp(rng.uniform(0, np.log(1200))))
        ld = int(np.exp(rng.uniform(0, np.log(3000))))
        if rng.random() < 0.05:
            lq = 0
        kind = rng.integers(0, 4)
        if kind == 0:
            q, d = rand_seq(rng, lq), rand_seq(rng, ld)
        elif kind == 1:  # mutated: db from the query
            q = synth.random_bases(int(rng.integers(1 << 30)), lq).tobytes()
            d = synth.mutate(q, float(rng.uniform(0.01, 0.2)), seed=int(rng.integers(1 << 30)))[:max(ld, 1)]
        elif kind == 2:  # two letters: many co-optimal parents
            q = bytes(rng.choice([65, 67], lq).astype(np.uint8))
            d = bytes(rng.choice([65, 67], ld).astype(np.uint8))
        else:  # with N
            q = bytes(rng.choice(list(b"ACGTN"), lq).astype(np.uint8))
            d = bytes(rng.choice(list(b"ACGTN"), ld).astype(np.uint8))
        out.append((q, d))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("seed", [1, 2, 3])
def test_mixed_shape_fuzz(saln, oracle, seed):
    pairs = _pairs(seed, 60)
    res, cig = saln.nw_align_batch([q for q, _ in pairs], [d for _, d in pairs],
                                   pairs=[(k, k) for k in range(len(pairs))])
    for k, (q, d) in enumerate(pairs):
        o = oracle.nw(q, d, literal_dfs=False)
        tag = (seed, k, len(q), len(d))
        assert int(res["score"][k]) == o.score, tag
        assert int(res["end_states"][k]) == o.end_states, tag
        assert (int(res["status"][k]) == 2) == o.panics, tag
        got = saln.cigar_ops_string(cig[k]) if res["printed"][k] else None
        assert got == o.first_ops, tag
