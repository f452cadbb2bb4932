set -e
B=tools/micro/hip_init_time
for rep in 1 2 3; do
for e in "X=1" "GPU_MAX_HW_QUEUES=1" "ROC_AQL_QUEUE_SIZE=4096" "HSA_KERNARG_POOL_SIZE=1048576" "ROC_SIGNAL_POOL_SIZE=64" "HIP_INITIAL_DM_SIZE=0" "HIP_FORCE_DEV_KERNARG=0" "HSA_ENABLE_SDMA=0"; do
  echo "== $e"; env $e timeout -k 5 30 $B | python3 -c "import sys,json; r=[json.loads(l) for l in sys.stdin if l.startswith('{\"step')]; print(' '.join(f'{x[\"step\"][:12]}={x[\"ms\"]}' for x in r[:4]))"
done; done
