#!/bin/bash
# A/B of experimental in-tree builds (libsaln_<v>.so): fill / traceback
# kernel durations under rocprofv3 --kernel-trace --stats on tools/prof_nw.py.
# usage: tools/exp_ab.sh v1 v2 ...   ("def" = libsaln.so)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
mkdir -p gpurun_out/ab
for v in "$@"; do
  lib=$PWD/sequencealigning_amd/libsaln.so
  [[ $v != def ]] && lib=$PWD/sequencealigning_amd/libsaln_$v.so
  SALN_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/ab/$v -o run --output-format csv -- python3 tools/prof_nw.py --reps 10 $EXTRA > gpurun_out/ab/$v.log 2>&1 || { echo "$v failed rc=$?"; tail -5 gpurun_out/ab/$v.log; exit 1; }
  echo "== $v"
  find gpurun_out/ab/$v -name "*kernel_stats.csv" -exec python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'saln' in r['Name']: print('  %-60s %6s calls avg %.4f ms' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e6))
" {} \;
done
