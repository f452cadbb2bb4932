#!/bin/bash
# Host-buffer path (bench.py's `host` leg): stage times (SALN_HOST_TIMING=1),
# the NW batch parity tests, then the leg's rate.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/host
leg() { timeout -k 10 120 python -c "import sys; sys.path.insert(0, '.'); import bench, sequencealigning_amd as saln; print(bench.leg_host(saln))"; }
SALN_HOST_TIMING=1 leg > gpurun_out/host/timing.log 2>&1 || { tail -20 gpurun_out/host/timing.log; exit 1; }
grep -E "scatter|descs|layout|plan  " gpurun_out/host/timing.log | tail -4
timeout -k 10 300 python -m pytest tests/test_nw_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread -k "golden or batch or c2_scale or long_gaps" > gpurun_out/host/tests.log 2>&1 || { tail -20 gpurun_out/host/tests.log; exit 1; }
tail -1 gpurun_out/host/tests.log
leg > gpurun_out/host/leg.log 2>&1 || { tail -20 gpurun_out/host/leg.log; exit 1; }
tail -1 gpurun_out/host/leg.log
