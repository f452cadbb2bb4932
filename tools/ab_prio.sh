#!/bin/bash
# Issue priorities of the C2 walk and fill (s_setprio): this tree vs
# experiment builds sequencealigning_amd/libsaln_<name>.so (LIBS, e.g.
# "prev"), pipelined and sequential steps, REPS alternations on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06; mkdir -p $O
: > $O/ab_prio.jsonl
for i in ${REPS:-1 2}; do
  for l in cur ${LIBS:-prev}; do
    lib=""; [ $l != cur ] && lib=sequencealigning_amd/libsaln_$l.so
    for pl in "--pipeline" ""; do
      SALN_LIB=$lib timeout -k 10 180 python tools/ab_c2.py $pl --tag ${l}${pl:+_pipe}_$i >> $O/ab_prio.jsonl 2>> $O/ab_prio.err || exit 1
    done
  done
done
cat $O/ab_prio.jsonl
