#!/bin/bash
# Row fill experiments: C4 fill time (walk codes and score-only) per build
# variant (def / rb4 / rb64 / ri: see Makefile) and columns per lane K.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/rows2
O=gpurun_out/rows2
timeout -k 10 300 python -u -m pytest tests/test_nw_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "stripes or cooperative or very_long or deadend" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for v in ${VS:-def rb4 rb64 ri}; do
  lib=$PWD/sequencealigning_amd/libsaln.so
  [[ $v != def ]] && lib=$PWD/sequencealigning_amd/libsaln_$v.so
  for k in ${KS:-1 2 4}; do
    SALN_LIB=$lib SALN_ROWS_K=$k timeout -k 10 120 python tools/bench_long.py --len 100000 --reps 3 > $O/c4_${v}_$k.log 2>&1 || { cat $O/c4_${v}_$k.log; exit 1; }
    SALN_LIB=$lib SALN_ROWS_K=$k timeout -k 10 120 python tools/bench_long.py --len 100000 --reps 3 --score-only > $O/c4so_${v}_$k.log 2>&1 || exit 1
    python3 - "$v" "$k" $O/c4_${v}_$k.log $O/c4so_${v}_$k.log <<'PY'
import json, sys
a = json.loads(open(sys.argv[3]).read().strip().splitlines()[-1])
b = json.loads(open(sys.argv[4]).read().strip().splitlines()[-1])
print(f"{sys.argv[1]:5s} K={sys.argv[2]} fill {a['fill_ms']:7.2f} walk {a['traceback_ms']:5.2f} exec {a['execute_ms']:7.2f} | score-only {b['fill_ms']:7.2f}  score {a['score']}")
PY
  done
done
