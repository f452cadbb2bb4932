set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
SALN_NARROW_GROUPS=1 timeout -k 10 600 python -u -m pytest tests/test_nw_gpu.py tests/test_nw_fuzz_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/nar_tests.log 2>&1 || { tail -30 gpurun_out/nar_tests.log; exit 1; }
tail -2 gpurun_out/nar_tests.log
for i in 1 2; do for n in 0 1; do
  SALN_NARROW_GROUPS=$n timeout -k 10 120 python bench.py --steps 20 --warmup 3 --legs none --no-cpu-baseline > gpurun_out/nar_$n.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/nar_$n.log').read().strip().splitlines()[-1]);r=d['roofline'];print($n, d['value'], r['kernel_avg_ms'], r['traceback_avg_ms'], d['verified'])"
done; done
