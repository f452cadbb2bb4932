#!/bin/bash
# PMC passes over tools/prof_nw.py (kernel-trace only with --pmc; no sys/runtime trace).
# usage: tools/pmc.sh [extra prof_nw.py args]; PMC_SETS overrides the counter passes
# (';'-separated).  A pass that fails on an unknown counter is skipped; a
# timeout / abort / segfault ends the script.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
OUT=gpurun_out/pmc
rm -rf $OUT
mkdir -p $OUT
SETS=${PMC_SETS:-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY;FETCH_SIZE;WRITE_SIZE;TCC_HIT_sum TCC_MISS_sum;GRBM_GUI_ACTIVE SQ_ACTIVE_INST_VALU SQ_INSTS_LDS"}
i=0
IFS=';' read -ra PASSES <<< "$SETS"
for ctrs in "${PASSES[@]}"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/p$i -o run -- python3 ${PMC_SCRIPT:-tools/prof_nw.py} "$@" > $OUT/p$i.log 2>&1
  rc=$?
  if [[ $rc -eq 124 || $rc -eq 134 || $rc -eq 137 || $rc -eq 139 ]]; then echo "pass $i ($ctrs) rc=$rc: stopping"; tail -20 $OUT/p$i.log; exit 1; fi
  if [[ $rc -ne 0 ]]; then echo "pass $i ($ctrs) failed rc=$rc (skipped)"; tail -5 $OUT/p$i.log; fi
done
python3 tools/pmc_summary.py $OUT
