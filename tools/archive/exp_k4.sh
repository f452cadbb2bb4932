set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/k4
for k in 2 4; do
  for so in "" "--score-only"; do
    SALN_ROWS_K=$k timeout -k 10 200 python tools/bench_long.py --len 100000 --reps 3 $so > gpurun_out/k4/k${k}${so}.log 2>&1 || { tail -20 gpurun_out/k4/k${k}${so}.log; exit 1; }
    echo "K=$k $so $(tail -1 gpurun_out/k4/k${k}${so}.log | cut -c1-300)"
  done
done
