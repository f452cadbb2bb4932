#!/bin/bash
# Round-6 GPU steps.  STAGES (space-separated, default "smoke tests bench"):
#   abxcd    C4 row fill, XCD-local stripe runs (nw.rows_xcd) vs dispatch order,
#            REPS alternations of tools/bench_long.py (walk codes and score-only)
#   abwalk   C2 step with this tree's walker vs sequencealigning_amd/libsaln_prev.so
#            (an earlier commit's build), sequential and pipelined, REPS alternations
#   abfull   c2_full step (full parent sets): table fill vs generic fill, REPS alternations
#   abtab    C2 step, table fill variants TABS (nw.pk_tab: 1 scale 2, 2 scale 4, 3 row profiles), REPS alternations
#   c2full   the c2_full leg alone (full 1 B/cell parent sets)
#   smoke    __graft_entry__.smoke()
#   tests    pytest -m gpu (TESTS= narrows it to files, KEXPR= to a -k expression)
#   chains   tools/micro/row_chains (row-fill chains per wave)
#   bench    bench.py --steps 20 --warmup 3 (BENCH_ARGS= extra args)
#   prof     rocprofv3 --kernel-trace --stats of the headline command (pipelined),
#            its fills split into co-run / alone by tools/trace_overlap.py
#   profseq  the same with --no-pipeline (every fill alone)
#   proflegs the same over tools/prof_legs.py
#   pmc      PMC passes (tools/pmc.sh) of the headline workload -> pmc_traffic.json
#   pmclegs  PMC passes over tools/prof_legs.py -> pmc_legs.json
#   pmcspans PMC of the c4_spans leg's span fills (one after another: --pmc
#            serializes kernels) -> pmc_c4_spans.json
#   pmcxcd   PMC traffic of the c4 leg with nw.rows_xcd=0 (stripes in dispatch
#            order) -> pmc_c4_xcd0.json
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r06
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 $O/$name.log; exit 1; }; }
for st in ${STAGES:-smoke tests bench}; do
  case $st in
    abxcd)
      for i in ${REPS:-1 2}; do
        for x in 0 1; do
          step xcd${x}_walk_$i 120 python tools/bench_long.py --len 100000 --reps 5 --opt nw.rows_xcd=$x
          tail -1 $O/xcd${x}_walk_$i.log
          step xcd${x}_so_$i 120 python tools/bench_long.py --len 100000 --reps 5 --score-only --opt nw.rows_xcd=$x
          tail -1 $O/xcd${x}_so_$i.log
        done
      done
      for x in 0 1; do
        for ns in 100 400 782; do
          step lag${x}_$ns 120 python tools/bench_long.py --len $((ns * 128)) --ldb 20000 --reps 5 --score-only --opt nw.rows_xcd=$x --opt nw.rows_k=2
          tail -1 $O/lag${x}_$ns.log
        done
      done ;;
    abwalk)  # the walker of this tree vs the one in sequencealigning_amd/libsaln_prev.so
      for i in ${REPS:-1 2}; do
        for lib in prev cur; do
          for pl in "" "--pipeline"; do
            tag=walk_${lib}${pl:+_pipe}_$i
            if [ $lib = prev ]; then
              SALN_LIB=sequencealigning_amd/libsaln_prev.so step $tag 180 python tools/ab_c2.py --tag $tag $pl
            else
              step $tag 180 python tools/ab_c2.py --tag $tag $pl
            fi
            tail -1 $O/$tag.log
          done
        done
      done ;;
    abtab)  # C2 table fill variants (nw.pk_tab values TABS), sequential and pipelined
      for i in ${REPS:-1 2}; do
        for t in ${TABS:-1 3}; do
          for pl in "" "--pipeline"; do
            tag=tab${t}${pl:+_pipe}_$i
            step $tag 180 python tools/ab_c2.py --tag $tag $pl --opt nw.pk_tab=$t
            tail -1 $O/$tag.log
          done
        done
      done ;;
    abfull)  # full-code plans: table fill (nw.pk_tab=3) vs the generic fill (0), REPS alternations
      for i in ${REPS:-1 2}; do
        for t in 0 3; do
          for pl in "" "--pipeline"; do
            tag=full${t}${pl:+_pipe}_$i
            step $tag 180 python tools/ab_c2.py --full --tag $tag $pl --opt nw.pk_tab=$t
            tail -1 $O/$tag.log
          done
        done
      done ;;
    abwfa2)  # corrected WFA: this tree vs sequencealigning_amd/libsaln_prev.so, REPS alternations
      for i in ${REPS:-1 2}; do
        SALN_LIB=sequencealigning_amd/libsaln_prev.so step wfa2_prev_$i 300 python tools/bench_wfa_affine.py --pairs 200000
        tail -1 $O/wfa2_prev_$i.log
        step wfa2_cur_$i 300 python tools/bench_wfa_affine.py --pairs 200000
        tail -1 $O/wfa2_cur_$i.log
      done ;;
    c2full) step c2full 400 python bench.py --steps 5 --warmup 2 --legs c2_full --no-cpu-baseline
            tail -1 $O/c2full.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['configs']['c2_full'])[:1500])" ;;
    chains) step chains 300 tools/micro/row_chains
            cat $O/chains.log ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
           tail -3 $O/smoke.log ;;
    tests) if [ -n "$KEXPR" ]; then
             step tests 1500 python -u -m pytest ${TESTS:-tests} -k "$KEXPR" -m gpu -x -v --timeout 300 --timeout-method thread
           else
             step tests 1500 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 300 --timeout-method thread
           fi
           tail -3 $O/tests.log ;;
    bench) step bench 600 python bench.py --steps 20 --warmup 3 $BENCH_ARGS
           tail -1 $O/bench.log | cut -c1-3000 ;;
    prof) step prof 600 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --legs none --no-cpu-baseline
          find $O/prof -name '*kernel_stats.csv' -exec head -12 {} \; | cut -c1-220
          python3 tools/trace_overlap.py $O/prof --out $O/prof_overlap.json ;;
    profseq) step profseq 600 rocprofv3 --kernel-trace --stats -d $O/profseq -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --legs none --no-cpu-baseline --no-pipeline
          find $O/profseq -name '*kernel_stats.csv' -exec head -12 {} \; | cut -c1-220
          python3 tools/trace_overlap.py $O/profseq --out $O/profseq_overlap.json ;;
    proflegs) step proflegs 900 rocprofv3 --kernel-trace --stats -d $O/proflegs -o run --output-format csv -- python3 tools/prof_legs.py
              find $O/proflegs -name '*kernel_stats.csv' -exec head -20 {} \; | cut -c1-220 ;;
    pmctab) PMC_SETS="SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU" step pmctab 600 bash tools/pmc.sh --opt-sets "${OPT_SETS:-nw.pk_tab=1;nw.pk_tab=2}"
           python3 tools/pmc_summary.py gpurun_out/pmc > $O/pmctab_summary.txt 2>&1; cp -r gpurun_out/pmc $O/pmctab_raw; head -60 $O/pmctab_summary.txt ;;
    pmcc2full) PMC_SCRIPT=tools/prof_legs.py PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU" step pmc_c2full 600 bash tools/pmc.sh --legs c2_full
           python3 tools/pmc_traffic.py gpurun_out/pmc $O/pmc_c2full.json r06 legs > /dev/null || exit 1 ;;
    pmc)   PMC_SETS=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"} step pmc 900 bash tools/pmc.sh
           python3 tools/pmc_traffic.py gpurun_out/pmc $O/pmc_traffic.json r06 nw > /dev/null || exit 1 ;;
    pmclegs) PMC_SCRIPT=tools/prof_legs.py PMC_SETS=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU"} step pmc_legs 1100 bash tools/pmc.sh --legs ${PROF_LEGS:-c2_full,c1,c3,c3_affine,c4,c5}
           python3 tools/pmc_traffic.py gpurun_out/pmc $O/pmc_legs.json r06 legs > /dev/null || exit 1 ;;
    pmcspans) PMC_SCRIPT=tools/prof_legs.py PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU" step pmc_spans 600 bash tools/pmc.sh --legs c4_spans
           python3 tools/pmc_traffic.py gpurun_out/pmc $O/pmc_c4_spans.json r06 legs > /dev/null || exit 1 ;;
    pmcxcd) PMC_SCRIPT=tools/prof_legs.py PMC_SETS="FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU" step pmc_xcd0 600 bash tools/pmc.sh --legs c4 --opt nw.rows_xcd=0
           python3 tools/pmc_traffic.py gpurun_out/pmc $O/pmc_c4_xcd0.json r06 legs > /dev/null || exit 1 ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
echo done
