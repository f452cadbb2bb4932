#!/bin/bash
# Round 4: 4-bit walk codes (option nw.nib_codes) and the 8 x 19 walk variant
# (nw.narrow_walk) against the byte codes of round 3, on the configs[1] step
# (tools/ab_c2.py), alternating on one box after the GPU tests (TESTS=...).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/nib
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 $O/$name.log; exit 1; }; }
for i in ${REPS:-1 2 3}; do
  step byte$i 120 python tools/ab_c2.py --tag byte --opt nw.nib_codes=0
  tail -1 $O/byte$i.log
  step nib$i 120 python tools/ab_c2.py --tag nib16x10
  tail -1 $O/nib$i.log
  step narrow$i 120 python tools/ab_c2.py --tag nib8x19 --opt nw.narrow_walk=1
  tail -1 $O/narrow$i.log
done
if [[ -n ${TESTS:-} ]]; then
  step tests 900 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread
  tail -2 $O/tests.log
fi
