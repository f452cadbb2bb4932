#!/bin/bash
# A/B of the packed fills' mask layout (SALN_PK_SKEW=1 skewed per-wave
# regions, 0 the interleaved row layout): packed-path GPU tests, then the C2
# bench alternating the two, twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/pkskew
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_nw_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread \
  -k "${TESTS_K:-not zzz}" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for v in ${VS:-1 0}; do
    SALN_PK_SKEW=$v timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --legs none > $O/b_$v.log 2>&1 || { tail -20 $O/b_$v.log; exit 1; }
    tail -1 $O/b_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('skew=$v', d['value'], d['ms_per_step'], 'fill', r['kernel_avg_ms'], 'tb', r['traceback_avg_ms'], d.get('verified'))"
  done
done
