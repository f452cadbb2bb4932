# nw.walk_waves A/B on the C2 headline workload (tools/ab_c2.py): this tree's
# library with the auto grid and explicit caps, against
# sequencealigning_amd/libsaln_prev.so (a lane per pair), pipelined and
# sequential, REPS alternations.
set -e
mkdir -p gpurun_out/r05
A="timeout -k 10 120 python tools/ab_c2.py"
for rep in ${REPS:-1 2}; do
  SALN_LIB=sequencealigning_amd/libsaln_prev.so $A --pipeline --tag prev > /tmp/o 2>&1; tail -1 /tmp/o
  for w in ${WAVES:--1 0 768 1024}; do
    $A --pipeline --opt nw.walk_waves=$w --tag ww$w > /tmp/o 2>&1; tail -1 /tmp/o
  done
  SALN_LIB=sequencealigning_amd/libsaln_prev.so $A --tag seq_prev > /tmp/o 2>&1; tail -1 /tmp/o
  $A --tag seq_auto > /tmp/o 2>&1; tail -1 /tmp/o
done
