#!/bin/bash
# A/B of the packed stripe fill (SALN_STRIPE_PK=1) against the default stripe
# fill: C4 and batches of 2 / 5 kbp pairs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
for pk in 0 1; do
  echo "== SALN_STRIPE_PK=$pk"
  SALN_STRIPE_PK=$pk timeout -k 10 120 python tools/bench_long.py --len 100000 --reps 2 || exit 1
  SALN_STRIPE_PK=$pk timeout -k 10 120 python tools/bench_long.py --len 100000 --reps 2 --score-only || exit 1
  SALN_STRIPE_PK=$pk timeout -k 10 200 python tools/bench_shapes.py --shape 2000x2000 --shape 5000x5000 --pairs 400 2>/dev/null || exit 1
done
