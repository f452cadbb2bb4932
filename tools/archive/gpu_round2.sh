#!/bin/bash
# Round-2 evidence: smoke, GPU tests, the full bench line (all configs), rocprofv3
# kernel stats of the headline (C2) command and of the C4 pair, batch shapes with
# the stripe fills, PMC traffic of the C2 fill.  Every GPU step has its own time
# limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r02
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -30 $O/$name.log; exit 1; }; }
[[ ${SKIP_TESTS:-0} == 1 ]] || {
  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
  tail -1 $O/tests.log
}
step bench 900 python bench.py --steps 20 --warmup 3
tail -1 $O/bench.log | cut -c1-600
step prof_c2 600 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --legs none
step prof_c4 600 rocprofv3 --kernel-trace --stats -d $O/prof_c4 -o run --output-format csv -- python3 tools/bench_long.py --len 100000 --reps 10
step shapes_a 600 python tools/bench_shapes.py --shape 2000x2000 --shape 5000x5000 --pairs 400
step shapes_b 600 python tools/bench_shapes.py --shape 1000x1000 --shape 600x600 --pairs 8000
SALN_STRIPE_PK=0 step shapes_c 600 python tools/bench_shapes.py --shape 2000x2000 --shape 5000x5000 --pairs 400
tail -n 2 $O/shapes_a.log $O/shapes_b.log $O/shapes_c.log
if [[ ${PMC:-1} == 1 ]]; then
  PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" step pmc 900 bash tools/pmc.sh
  python3 tools/pmc_traffic.py gpurun_out/pmc $O/pmc_traffic.json r02 > /dev/null || exit 1
fi
echo done
