#!/bin/bash
# GPU session for the corrected gap-affine WFA: parity tests, then the
# configs[2]-shaped bench (tools/bench_wfa_affine.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_wfa_affine_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_wfa2.log 2>&1 || { tail -40 gpurun_out/pytest_wfa2.log; exit 1; }
tail -3 gpurun_out/pytest_wfa2.log
timeout -k 10 600 python tools/bench_wfa_affine.py --pairs "${WFA2_PAIRS:-20000}" --distinct 1000 --reps 2 > gpurun_out/wfa2.log 2>&1 || { tail -5 gpurun_out/wfa2.log; exit 1; }
tail -1 gpurun_out/wfa2.log
