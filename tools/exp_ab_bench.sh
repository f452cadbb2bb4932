#!/bin/bash
# A/B of the in-tree build against libsaln_base.so (the previous commit's
# kernels, built by hand for the experiment), alternating on one box, after
# the GPU tests of the new build.  Not part of the product.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/${AB_OUT:-ab}
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -30 $O/$name.log; exit 1; }; }
[[ ${SKIP_TESTS:-0} == 1 ]] || { step tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread; tail -1 $O/tests.log; }
for i in 1 2 3; do
  SALN_LIB=$PWD/sequencealigning_amd/libsaln_base.so step base$i 300 python bench.py --steps 40 --warmup 5 --legs none --no-cpu-baseline
  step new$i 300 python bench.py --steps 40 --warmup 5 --legs none --no-cpu-baseline
done
for f in base1 new1 base2 new2 base3 new3; do python3 -c "import json; d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1]); print('$f', d['value'], d['ms_per_step'], d['roofline']['kernel_avg_ms'], d['roofline']['traceback_avg_ms'], d.get('verified'))"; done
echo done
