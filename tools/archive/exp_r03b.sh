#!/bin/bash
# Round-3 A/B: the packed fill's steady-state steps (SALN_PK_STEADY=0 / 1),
# after the full GPU suite; three alternations on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/exp
mkdir -p $O
t() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -30 $O/$name.log; exit 1; }; }
t tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 $O/tests.log
for i in 1 2 3; do
  for n in 0 1; do
    SALN_PK_STEADY=$n t st_$n 120 python bench.py --steps 20 --warmup 3 --legs none --no-cpu-baseline
    python -c "import json;d=json.loads(open('$O/st_$n.log').read().strip().splitlines()[-1]);r=d['roofline'];print('steady', $n, d['value'], r['kernel_avg_ms'], r['traceback_avg_ms'], d['verified']['mismatches'])"
  done
done
