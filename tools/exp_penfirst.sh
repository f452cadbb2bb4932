# A/B: score-only packed fill with the row's penalties first (in-tree) vs
# per column (libsaln_pf0.so), on the configs[4] slice; alternated twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for i in 1 2; do
  for tag in base pf0; do
    if [ $tag = pf0 ]; then lib=$PWD/sequencealigning_amd/libsaln_pf0.so; else lib=; fi
    SALN_LIB=$lib timeout -k 10 120 python tools/bench_avsa.py --nq 1000 --ndb 100000 --reps 3 > gpurun_out/pf_${tag}_$i.log 2>&1 || exit 1
    echo "$tag $i $(tail -1 gpurun_out/pf_${tag}_$i.log | cut -c1-200)"
  done
done
