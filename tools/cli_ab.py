"""A/B of saln CLI invocations on bench.py's cli workload (316 x 316 FASTA
records of 150 bp G-iid, seed 0x5EED0002; tools only): each argument set
runs REPS times, alternating, stdout to a file; prints the walls.

    python tools/cli_ab.py [--reps 3] -- "--chunk-pairs 65536" "--chunk-pairs 16384"
"""
import argparse
import json
import os
import shlex
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--n", type=int, default=316)
    ap.add_argument("sets", nargs="+")
    a = ap.parse_args()
    from sequencealigning_amd import synth
    n = a.n
    qs, qo, ds, do = synth.iid_pairs(n, 150, 150, seed=0x5EED0002)
    cli = os.path.join(ROOT, "sequencealigning_amd", "saln")
    with tempfile.TemporaryDirectory() as t:
        qf, df, of = (os.path.join(t, x) for x in ("q.fa", "d.fa", "out.txt"))
        for path, s, o, tag in ((qf, qs, qo, b"q"), (df, ds, do, b"d")):
            with open(path, "wb") as fh:
                for k in range(n):
                    fh.write(b">%s%d\n%s\n" % (tag, k, s[int(o[k]):int(o[k + 1])].tobytes()))
        base = [cli, "-q", qf, "-d", df, "-a", "needleman-wunsch", "--no-timing", "--no-abort",
                "--max-blocks", "1"]
        walls = {x: [] for x in a.sets}
        for _ in range(a.reps):
            for x in a.sets:
                with open(of, "wb") as out:
                    t0 = time.perf_counter()
                    r = subprocess.run(base + shlex.split(x), stdout=out, stderr=subprocess.PIPE,
                                       timeout=300)
                    walls[x].append(round(time.perf_counter() - t0, 4))
                if r.returncode:
                    raise SystemExit(f"{x}: exit {r.returncode} {r.stderr[-400:]!r}")
        cells = n * n * 150 * 150
        for x, w in walls.items():
            print(json.dumps({"args": x, "walls_s": w,
                              "gcups_best": round(cells / min(w) / 1e9, 2)}))


if __name__ == "__main__":
    main()
