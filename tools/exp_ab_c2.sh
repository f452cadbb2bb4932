#!/bin/bash
# A/B of the in-tree build against experiment builds made by hand for the
# experiment (sequencealigning_amd/libsaln_<tag>.so; AB_TAGS, default "base":
# the previous commit's kernels), alternating on one box (tools/ab_c2.py),
# after the GPU tests of the new build.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/ab
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -30 $O/$name.log; exit 1; }; }
[[ ${SKIP_TESTS:-0} == 1 ]] || { step tests 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread; tail -1 $O/tests.log; }
for i in 1 2 3; do
  for tag in ${AB_TAGS:-base}; do
    SALN_LIB=$PWD/sequencealigning_amd/libsaln_$tag.so step ${tag}$i 120 python tools/ab_c2.py --tag $tag
    tail -1 $O/${tag}$i.log
  done
  step new$i 120 python tools/ab_c2.py --tag new
  tail -1 $O/new$i.log
done
