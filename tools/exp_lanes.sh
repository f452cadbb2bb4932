#!/bin/bash
# A/B of the i32-lanes fill (shapes past the packed reach) against libsaln_base.so, after the GPU tests.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
set -o pipefail
O=gpurun_out/lanes; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for i in 1 2; do
  SALN_LIB=$PWD/sequencealigning_amd/libsaln_base.so timeout -k 10 300 python tools/bench_shapes.py --shape 150x5000 --shape 100x6000 --pairs 4000 > $O/base$i.log 2>&1 || exit 1
  timeout -k 10 300 python tools/bench_shapes.py --shape 150x5000 --shape 100x6000 --pairs 4000 > $O/new$i.log 2>&1 || exit 1
done
tail -n 2 $O/base1.log $O/new1.log $O/base2.log $O/new2.log
