#!/bin/bash
# Round-3 A/B: (1) 8 x 19 lane groups for <= 152-column queries with the
# 20-byte-segment LDS walker (SALN_NARROW_GROUPS=1); (2) the row fill's coder
# wave (SALN_ROWS_SPLIT=1).  Parity first (the GPU tests that cover each),
# then two alternations of each timing on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/exp
mkdir -p $O
t() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -30 $O/$name.log; exit 1; }; }
SALN_NARROW_GROUPS=1 t nar_tests 600 python -u -m pytest tests/test_nw_gpu.py tests/test_nw_fuzz_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 $O/nar_tests.log
SALN_ROWS_SPLIT=1 t split_tests 600 python -u -m pytest tests/test_nw_gpu.py tests/test_robustness_gpu.py tests/test_cli_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 $O/split_tests.log
for i in 1 2; do
  for n in 0 1; do
    SALN_NARROW_GROUPS=$n t nar_$n 120 python bench.py --steps 20 --warmup 3 --legs none --no-cpu-baseline
    python -c "import json;d=json.loads(open('$O/nar_$n.log').read().strip().splitlines()[-1]);r=d['roofline'];print('narrow', $n, d['value'], r['kernel_avg_ms'], r['traceback_avg_ms'], d['verified']['mismatches'])"
  done
  for n in 0 1; do
    SALN_ROWS_SPLIT=$n t split_$n 300 python bench.py --steps 1 --warmup 1 --legs c4,c1 --no-cpu-baseline
    python -c "import json;d=json.loads(open('$O/split_$n.log').read().strip().splitlines()[-1]);c=d['configs'];print('split', $n, c['c4']['gpu']['fill_ms'], c['c4']['gpu']['execute_ms'], c['c1']['gpu']['fill_ms'], c['c1']['gpu']['execute_ms'])"
  done
done
