#!/bin/bash
# Walker time against the pair count (C2 shape): the latency floor (few waves)
# against the throughput regime (tools/ab_c2.py, one box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out/wk
for n in 12500 25000 50000 100000 200000 400000; do
  timeout -k 10 120 python tools/ab_c2.py --pairs $n --steps 20 --tag p$n > gpurun_out/wk/p$n.log 2>&1 || { tail -20 gpurun_out/wk/p$n.log; exit 1; }
  tail -1 gpurun_out/wk/p$n.log
done
