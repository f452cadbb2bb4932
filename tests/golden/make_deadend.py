"""Regenerates tests/golden/nw_deadend.json: pairs past the sentinel line
(a side longer than ~5,460 with the default scoring) whose reference DFS meets
sentinel-rooted subtrees - M[0][j], I[0][j], M[i][0], D[i][0] have no parents
and are dropped silently (needleman_wunsch_affine.rs:172-216, :281-329).
Expected values come from both oracles (oracle/refcpu.c full matrices +
memoised DFS, oracle/reflinear.c parent sets + literal DFS), which must agree;
`dead` counts the (cell, state) nodes the DFS exhausted before its first
event.  Run from the repo root: python tests/golden/make_deadend.py"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
from oracle import refcpu  # noqa: E402


def draw(rng, alpha, n):
    a = np.frombuffer(alpha, np.uint8)
    return a[rng.integers(0, len(a), n)].tobytes()


def cases():
    # search 1: the first pairs of a seeded sweep over sentinel-region shapes
    rng = np.random.default_rng(0)
    shapes = [(5600, 150), (150, 5600), (5500, 300), (300, 5520), (6000, 1000), (5470, 40),
              (45, 5470), (5465, 2)]
    alphas = [b"ACGT", b"AC", b"A", b"AAAC"]
    for k in range(40):
        lq, ld = shapes[k % 8]
        al = alphas[k % 4]
        q, d = draw(rng, al, lq), draw(rng, al, ld)
        if k in (7, 11, 12, 24, 36, 39):  # all-dead, panics, printed after a dead subtree
            yield f"sweep{k}", q, d
    # search 3: near the sentinel crossover (D[0][5459] == -32768)
    rng = np.random.default_rng(5000 + 111)
    lq, ld = int(rng.integers(5455, 5475)), int(rng.integers(1, 12))
    lq, ld = ld, lq
    yield "cross111", draw(rng, b"AC", lq), draw(rng, b"AC", ld)


def main():
    out = []
    for name, q, d in cases():
        o = refcpu.nw(q, d, literal_dfs=False)
        sc, es, pan, first, dead = refcpu.nw_first_linear(q, d, threads=4)
        assert (sc, es, pan, first) == (o.score, o.end_states, o.panics, o.first_ops), name
        out.append({"id": name, "query": q.decode(), "db": d.decode(), "score": sc,
                    "end_states": es, "panics": pan, "first_ops": first, "dead": dead})
        print(name, len(q), len(d), sc, pan, first is not None, dead)
    with open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "nw_deadend.json"), "w") as f:
        json.dump({"generator": "tests/golden/make_deadend.py", "pairs": out}, f)


if __name__ == "__main__":
    main()
