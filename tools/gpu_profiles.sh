#!/bin/bash
# Round-end evidence: smoke, GPU tests, bench, rocprofv3 kernel-trace stats of
# the bench command, PMC HBM traffic of the fill (FETCH_SIZE / WRITE_SIZE in
# separate passes), long-pair / WFA / all-vs-all tool lines.  Each GPU step is
# time-limited; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/final
O=gpurun_out/final
bash tools/gpu_round.sh smoke || exit 1
bash tools/gpu_round.sh test || exit 1
timeout -k 10 600 python bench.py --steps 20 --warmup 3 > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
tail -1 $O/bench.log
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
tail -1 $O/prof.log
PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU" bash tools/pmc.sh > $O/pmc.log 2>&1 || { tail -20 $O/pmc.log; exit 1; }
python3 tools/pmc_traffic.py gpurun_out/pmc $O/pmc_traffic.json > /dev/null || exit 1
cat $O/pmc_traffic.json
timeout -k 10 300 python tools/bench_long.py --len 1000 --reps 5 > $O/long1k.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_long.py --len 100000 --reps 2 > $O/long100k.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_long.py --len 100000 --reps 2 --score-only > $O/long100k_so.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_wfa.py --pairs 1000000 --reps 3 > $O/wfa.log 2>&1 || exit 1
timeout -k 10 600 python tools/bench_wfa_affine.py --pairs 100000 --distinct 2000 --reps 2 > $O/wfa_affine.log 2>&1 || exit 1
timeout -k 10 300 python tools/bench_avsa.py > $O/avsa.log 2>&1 || exit 1
for f in long1k long100k long100k_so wfa wfa_affine avsa; do echo "$f: $(tail -1 $O/$f.log | cut -c1-400)"; done
