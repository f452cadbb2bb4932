#!/bin/bash
# WFA kernel A/B: GPU WFA tests of the in-tree build, then bench legs (LEGS,
# default c3) through tools/ab_legs.py for sequencealigning_amd/libsaln_<tag>.so
# (AB_TAGS, default "old") and the in-tree build, alternating on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/wfa
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -30 $O/$name.log; exit 1; }; }
[[ ${SKIP_TESTS:-0} == 1 ]] || { step tests 600 python -u -m pytest tests/test_wfa_gpu.py tests/test_cli_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread; tail -1 $O/tests.log; }
for i in 1 2; do
  for tag in ${AB_TAGS:-old}; do
    SALN_LIB=$PWD/sequencealigning_amd/libsaln_$tag.so step $tag$i 300 python tools/ab_legs.py --legs ${LEGS:-c3} --tag $tag
    grep '^{' $O/$tag$i.log
  done
  step new$i 300 python tools/ab_legs.py --legs ${LEGS:-c3} --tag new
  grep '^{' $O/new$i.log
done
