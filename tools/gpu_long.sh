set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
bash tools/gpu_round.sh test || exit 1
timeout -k 10 300 python tools/bench_long.py --len 1000 --reps 5 > gpurun_out/long1k.log 2>&1 || { tail -5 gpurun_out/long1k.log; exit 1; }
tail -2 gpurun_out/long1k.log
timeout -k 10 300 python tools/bench_long.py --len 100000 --reps 2 > gpurun_out/long100k.log 2>&1 || { tail -5 gpurun_out/long100k.log; exit 1; }
tail -2 gpurun_out/long100k.log
timeout -k 10 300 python tools/bench_long.py --len 100000 --reps 2 --score-only > gpurun_out/long100k_so.log 2>&1 || { tail -5 gpurun_out/long100k_so.log; exit 1; }
tail -2 gpurun_out/long100k_so.log
