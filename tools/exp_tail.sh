set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for n in 100000 98304 90112 106496 114688 131072; do
  timeout -k 10 120 python bench.py --steps 20 --warmup 3 --legs none --no-cpu-baseline --pairs $n > gpurun_out/tail_$n.log 2>&1 || exit 1
  python - "$n" <<'PY'
import json,sys
n=sys.argv[1]; d=json.loads(open(f"gpurun_out/tail_{n}.log").read().strip().splitlines()[-1])
r=d["roofline"]; print(n, d["value"], d["ms_per_step"], r["kernel_avg_ms"], round(r["kernel_avg_ms"]*1e6/int(n),3), "ns/pair fill", d.get("walk_ms", d.get("traceback_ms")))
PY
done
