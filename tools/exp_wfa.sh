#!/bin/bash
# WFA (reference semantics) kernel A/B: GPU WFA tests, then configs[2]-shaped
# legs through tools/ab_legs.py for the in-tree build and
# sequencealigning_amd/libsaln_old.so (the previous kernels), alternating.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/wfa
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -30 $O/$name.log; exit 1; }; }
step tests 600 python -u -m pytest tests/test_wfa_gpu.py tests/test_cli_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread
tail -1 $O/tests.log
for i in 1 2; do
  SALN_LIB=$PWD/sequencealigning_amd/libsaln_old.so step old$i 300 python tools/ab_legs.py --legs ${LEGS:-c3} --tag old
  grep '^{' $O/old$i.log
  step new$i 300 python tools/ab_legs.py --legs ${LEGS:-c3} --tag new
  grep '^{' $O/new$i.log
done
