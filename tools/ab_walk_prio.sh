# Experiment record: needs a build whose walker takes s_setprio from an option
# "nw.walk_prio" (not shipped: priority 3/2/1/0 measured within 0.3 %,
# profiles/r05_walk_prio_ab.jsonl).
set -e
A="timeout -k 10 120 python tools/ab_c2.py --pipeline"
for rep in 1 2; do
  SALN_LIB=sequencealigning_amd/libsaln_prev.so $A --tag prev > /tmp/o 2>&1; tail -1 /tmp/o
  for pr in 3 2 1 0; do $A --opt nw.walk_prio=$pr --tag prio$pr > /tmp/o 2>&1; tail -1 /tmp/o; done
done
