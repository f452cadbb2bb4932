"""A/B of saln CLI invocations on bench.py's cli workload (316 x 316 FASTA
records of 150 bp G-iid, seed 0x5EED0002; tools only): each argument set
runs REPS times, alternating, stdout to a file; prints the walls.

    python tools/cli_ab.py [--reps 3] -- "--chunk-pairs 65536" "--chunk-pairs 16384"
    python tools/cli_ab.py --stages --outdir /dev/shm -- "" "--teardown"
(leading NAME=VALUE tokens of a set are environment variables of its runs)
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
    ap.add_argument("--outdir", default=None, help="directory of the output file (e.g. /dev/shm)")
    ap.add_argument("--stages", action="store_true", help="add --stage-times; print each run's "
                    "context / render / print stages")
    ap.add_argument("sets", nargs="+")
    a = ap.parse_args()
    from sequencealigning_amd import synth
    n = a.n
    qs, qo, ds, do = synth.iid_pairs(n, 150, 150, seed=0x5EED0002)
    cli = os.path.join(ROOT, "sequencealigning_amd", "saln")
    with tempfile.TemporaryDirectory() as t:
        qf, df = (os.path.join(t, x) for x in ("q.fa", "d.fa"))
        of = os.path.join(a.outdir or t, f"cli_ab_{os.getpid()}.txt")
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
                    t0, c0 = time.perf_counter(), time.time_ns()
                    toks = shlex.split(x)  # leading NAME=VALUE tokens: environment
                    env = dict(os.environ)
                    while toks and "=" in toks[0] and not toks[0].startswith("-"):
                        k, v = toks.pop(0).split("=", 1)
                        env[k] = v
                    r = subprocess.run(base + toks + (["--stage-times"] if a.stages else []),
                                       stdout=out, stderr=subprocess.PIPE, timeout=300, env=env)
                    walls[x].append(round(time.perf_counter() - t0, 4))
                    c1 = time.time_ns()
                if a.stages:
                    keep = ("context", "render batch", "print", "exit", "load fasta")
                    st = {}
                    for ln in r.stderr.decode("latin-1").splitlines():
                        if ln.startswith("[saln-clock] main-entry"):
                            st["before main"] = round((int(ln.split()[-1]) - c0) / 1e6, 2)
                        if ln.startswith("[saln-clock] main-exit"):
                            st["after main"] = round((c1 - int(ln.split()[-1])) / 1e6, 2)
                        if ln.startswith("[saln "):
                            name, ms = ln.split("]", 1)[1].rsplit(None, 2)[0].strip(), ln.split()[-2]
                            if name.startswith(keep):
                                st[name] = round(st.get(name, 0.0) + float(ms), 2)
                    print(json.dumps({"args": x, "wall_s": walls[x][-1], "stages_ms": st}), flush=True)
                os.remove(of)
                if r.returncode:
                    raise SystemExit(f"{x}: exit {r.returncode} {r.stderr[-400:]!r}")
        cells = n * n * 150 * 150
        for x, w in walls.items():
            print(json.dumps({"args": x, "walls_s": w,
                              "gcups_best": round(cells / min(w) / 1e9, 2)}))


if __name__ == "__main__":
    main()
