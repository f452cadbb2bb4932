set -o pipefail
for v in ${VARS:-def p16 p8 def}; do
  lib=$PWD/sequencealigning_amd/libsaln.so; [[ $v != def ]] && lib=$PWD/sequencealigning_amd/libsaln_$v.so
  for L in 1000 100000; do
    r=3; [[ $L == 1000 ]] && r=50
    echo -n "$v $L "; SALN_LIB=$lib timeout -k 10 120 python tools/bench_long.py --len $L --reps $r || exit 1
  done
  echo -n "$v so "; SALN_LIB=$lib timeout -k 10 120 python tools/bench_long.py --len 100000 --reps 3 --score-only || exit 1
done
