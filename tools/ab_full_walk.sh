set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
O=gpurun_out/r06; mkdir -p $O
: > $O/ab_full_walk.jsonl
for i in 1 2; do
  for w in 0 -1; do
    for pl in "" "--pipeline"; do
      timeout -k 10 180 python tools/ab_c2.py --full --tag fullw${w}${pl:+_pipe}_$i $pl --opt nw.walk_waves=$w >> $O/ab_full_walk.jsonl 2> $O/ab_full_walk.err || exit 1
    done
  done
done
timeout -k 10 600 python -u -m pytest tests/test_nw_gpu.py -m gpu -k "full or walk_waves or bail" -x -q --timeout 300 --timeout-method thread > $O/tests_fw.log 2>&1; tail -2 $O/tests_fw.log
