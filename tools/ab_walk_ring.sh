#!/bin/bash
# Walker window depth (WalkGeo::W, slots per window) for the 4-bit walk: this
# tree (W = 4) vs experiment builds with other depths (WS="4 6 8": the
# libraries sequencealigning_amd/libsaln_w<W>.so, each built with WalkGeo's W
# changed), sequential and pipelined C2 steps, REPS alternations on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06; mkdir -p $O
: > $O/ab_walk_ring.jsonl
for i in ${REPS:-1 2}; do
  for w in ${WS:-4 6 8}; do
    lib=""; [ $w != 4 ] && lib=sequencealigning_amd/libsaln_w$w.so
    for pl in "" "--pipeline"; do
      SALN_LIB=$lib timeout -k 10 180 python tools/ab_c2.py $pl --tag w${w}${pl:+_pipe}_$i >> $O/ab_walk_ring.jsonl 2>> $O/ab_walk_ring.err || exit 1
    done
  done
done
cat $O/ab_walk_ring.jsonl
