#!/bin/bash
# A/B of the LLVM scheduling strategy nw_kernels.hip is built with
# (libsaln_<v>.so, `-mllvm -amdgpu-sched-strategy=...`):
# the C2 bench alternating the libraries, twice.  LIBS: space-separated
# suffixes ("" = libsaln.so).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/sched
mkdir -p $O
for rep in 1 2; do
  for v in ${LIBS:-def s1 s3 s4}; do
    lib=sequencealigning_amd/libsaln.so
    [ "$v" != def ] && lib=sequencealigning_amd/libsaln_$v.so
    SALN_LIB=$PWD/$lib timeout -k 10 200 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --legs none $EXTRA > $O/b_$v.log 2>&1 || { tail -20 $O/b_$v.log; exit 1; }
    tail -1 $O/b_$v.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$v', d['value'], d['ms_per_step'], 'fill', r['kernel_avg_ms'], 'tb', r['traceback_avg_ms'], d.get('verified'))"
  done
done
