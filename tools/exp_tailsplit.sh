# A/B: C2 with the tail sub-batch split (default) vs SALN_TAIL_SPLIT=0, two
# alternations on one box (bench.py headline only).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2; do
  for ts in 1 0; do
    SALN_TAIL_SPLIT=$ts timeout -k 10 120 python bench.py --steps 30 --warmup 5 --legs none --no-cpu-baseline > gpurun_out/ts_${ts}_$i.log 2>&1 || exit 1
    python - "$ts" "$i" <<'PY'
import json, sys
d = json.loads(open(f"gpurun_out/ts_{sys.argv[1]}_{sys.argv[2]}.log").read().strip().splitlines()[-1])
print("split" if sys.argv[1] == "1" else "nosplit", sys.argv[2], d["value"], d["ms_per_step"], d["roofline"]["kernel_avg_ms"], d.get("verified"))
PY
  done
done
