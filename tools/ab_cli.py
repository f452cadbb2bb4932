"""A/B of the drop-in CLI's process wall time under engine option sets
(`saln --option NAME=VALUE`), alternated run by run on one box.

The inputs are bench.py's `cli` / `cli_all` legs' FASTA files (316 x 316
records of 150 bp, G-iid or G-mut(5 %) copies of one base); stdout goes to
/dev/null as in those legs. Each run also records its `--stage-times` lines
(stderr), so a change in one stage (context, the first chunk's copies) can be
told from noise in the others.

    python tools/ab_cli.py --sets "host.warmup=0;host.warmup=1" --reps 8 [--all-blocks]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--sets", required=True, help="';'-separated option sets, each 'k=v,k=v' or ''")
    ap.add_argument("--reps", type=int, default=8)
    ap.add_argument("--n", type=int, default=316)
    ap.add_argument("--all-blocks", action="store_true", help="cli_all's G-mut records, every block")
    ap.add_argument("--tag", default="")
    a = ap.parse_args()
    from sequencealigning_amd import synth
    seed, L = 0x5EED0002, 150
    if a.all_blocks:
        rng = np.random.default_rng(seed)
        base = bytes(rng.choice(np.frombuffer(b"ACGT", np.uint8), L))
        q = [synth.mutate(base, 0.05, seed=seed + k) for k in range(a.n)]
        d = [synth.mutate(base, 0.05, seed=seed + a.n + k) for k in range(a.n)]
    else:
        qs, qo, ds, do = synth.iid_pairs(a.n, L, L, seed=seed)
        q = [qs[int(qo[k]):int(qo[k + 1])].tobytes() for k in range(a.n)]
        d = [ds[int(do[k]):int(do[k + 1])].tobytes() for k in range(a.n)]
    cli = os.path.join(ROOT, "sequencealigning_amd", "saln")
    sets = [s.strip() for s in a.sets.split(";")]
    walls = {s: [] for s in sets}
    stages = {s: {} for s in sets}
    with tempfile.TemporaryDirectory() as tdir:
        qf, df = os.path.join(tdir, "q.fa"), os.path.join(tdir, "d.fa")
        for path, recs, tag in ((qf, q, "q"), (df, d, "d")):
            with open(path, "wb") as fh:
                for k, r in enumerate(recs):
                    fh.write(b">%s%d\n%s\n" % (tag.encode(), k, r))
        base_cmd = [cli, "-q", qf, "-d", df, "-a", "needleman-wunsch", "--no-timing", "--no-abort",
                    "--stage-times"]
        if not a.all_blocks:
            base_cmd += ["--max-blocks", "1"]
        # one untimed run pages the library and the files in
        subprocess.run(base_cmd, stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL, timeout=120,
                       check=True)
        for rep in range(a.reps):
            for s in sets:
                cmd = list(base_cmd)
                for kv in filter(None, s.split(",")):
                    cmd += ["--option", kv]
                with open(os.devnull, "wb") as out:
                    t0 = time.perf_counter()
                    r = subprocess.run(cmd, stdout=out, stderr=subprocess.PIPE, timeout=120)
                    w = time.perf_counter() - t0
                if r.returncode != 0:
                    raise RuntimeError(f"{cmd}: exit {r.returncode}: {r.stderr[-400:]!r}")
                walls[s].append(w)
                seen = {}
                for ln in r.stderr.decode("latin-1").splitlines():
                    if not ln.startswith("[saln "):
                        continue
                    body = ln.split("]", 1)[1].strip()
                    name, _, val = body.rpartition(" ")
                    name = name.strip()
                    if val == "ms" and " " in name:
                        name, val = name.rsplit(" ", 1)[0].strip(), name.rsplit(" ", 1)[1]
                    try:
                        ms = float(val)
                    except ValueError:
                        continue
                    k = seen.get(name, 0)
                    seen[name] = k + 1
                    if k == 0:  # first occurrence: the first chunk's stage
                        stages[s].setdefault(name, []).append(ms)
    for s in sets:
        st = {k: round(float(np.median(v)), 3) for k, v in stages[s].items()
              if k in ("context", "plan: pairs h2d", "render: execute", "render batch", "print")}
        print(json.dumps({"tag": a.tag, "set": s or "defaults", "all_blocks": a.all_blocks,
                          "wall_s_median": round(float(np.median(walls[s])), 4),
                          "wall_s_min": round(min(walls[s]), 4),
                          "walls_s": [round(x, 3) for x in walls[s]],
                          "first_chunk_stage_ms_median": st}), flush=True)


if __name__ == "__main__":
    main()
