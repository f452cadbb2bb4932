#!/bin/bash
# Row-synchronous stripe fill: parity of the stripe paths, then C4 / C1 timing
# for SALN_ROWS_K = 0 (skewed stripes), 1, 2, 4.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/rows
O=gpurun_out/rows
timeout -k 10 400 python -u -m pytest tests/test_nw_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread \
  -k "stripes or cooperative or very_long or deadend or degenerate or random_shapes or mutated" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -2 $O/tests.log
for k in ${KS:-0 1 2 4}; do
  SALN_ROWS_K=$k timeout -k 10 120 python tools/bench_long.py --len 100000 --reps 3 > $O/c4_k$k.log 2>&1 || { cat $O/c4_k$k.log; exit 1; }
  SALN_ROWS_K=$k timeout -k 10 120 python tools/bench_long.py --len 100000 --reps 3 --score-only > $O/c4so_k$k.log 2>&1 || exit 1
  SALN_ROWS_K=$k timeout -k 10 120 python tools/bench_long.py --len 1000 --reps 20 > $O/c1_k$k.log 2>&1 || exit 1
  echo "K=$k c4: $(tail -1 $O/c4_k$k.log)"
  echo "K=$k c4so: $(tail -1 $O/c4so_k$k.log)"
  echo "K=$k c1: $(tail -1 $O/c1_k$k.log)"
done
