#!/bin/bash
# Round-3 GPU steps.  STAGES (space-separated, default "smoke tests bench"):
#   smoke  __graft_entry__.smoke()
#   tests  pytest -m gpu (TESTS= narrows it: a path or -k expression args)
#   bench  bench.py --steps 20 --warmup 3 (BENCH_ARGS= extra args)
#   prof   rocprofv3 --kernel-trace --stats of the headline command
#   proflegs  the same over tools/prof_legs.py (the legs' GPU workloads)
#   pmc    PMC passes (tools/pmc.sh) of the headline workload -> pmc_traffic.json
#   pmclegs   PMC passes over tools/prof_legs.py -> pmc_legs.json
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r03
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 $O/$name.log; exit 1; }; }
for st in ${STAGES:-smoke tests bench}; do
  case $st in
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step tests 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread
           tail -3 $O/tests.log ;;
    bench) step bench 900 python bench.py --steps 20 --warmup 3 $BENCH_ARGS
           tail -1 $O/bench.log | cut -c1-900 ;;
    prof)  step prof_c2 600 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --legs none ;;
    proflegs) step prof_legs 900 rocprofv3 --kernel-trace --stats -d $O/prof_legs -o run --output-format csv -- python3 tools/prof_legs.py --legs ${PROF_LEGS:-c1,c3,c3_affine,c4,c5} ;;
    pmc)   PMC_SETS=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"} step pmc 900 bash tools/pmc.sh
           python3 tools/pmc_traffic.py gpurun_out/pmc $O/pmc_traffic.json r03 nw > /dev/null || exit 1 ;;
    pmclegs) PMC_SCRIPT=tools/prof_legs.py PMC_SETS=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU"} step pmc_legs 1100 bash tools/pmc.sh --legs ${PROF_LEGS:-c1,c3,c3_affine,c4,c5}
           python3 tools/pmc_traffic.py gpurun_out/pmc $O/pmc_legs.json r03 legs > /dev/null || exit 1 ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
echo done
