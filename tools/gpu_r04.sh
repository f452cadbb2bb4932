#!/bin/bash
# Round-4 GPU steps.  STAGES (space-separated, default "smoke tests bench"):
#   ab       A/B of the walk-code formats on the configs[1] step (tools/ab_c2.py;
#            AB= "tag:opts,..." overrides; REPS alternations)
#   cumap    tools/cu_map.py -> $O/cu_map.json
#   pipe     tools/cu_pipeline.py over walk-CU counts / layouts (PIPE_CASES)
#   pipetrace  rocprofv3 --kernel-trace of one pipeline case (PIPE_TRACE args)
#   rowfloor tools/micro/row_pk_floor (C4 row-step floor: i32 K=2 vs i16x2 frames)
#   spans    tools/spans_sweep.py over SPAN_CASES (spans:band_rows:edge_masks)
#   abpipe   bench headline --no-pipeline vs pipelined (default), REPS alternations
#   spanq    span counts under GPU_MAX_HW_QUEUES=4 and 16
#   clileg   bench.py's cli leg alone (with its stage breakdown)
#   smoke    __graft_entry__.smoke()
#   tests    pytest -m gpu (TESTS= narrows it)
#   bench    bench.py --steps 20 --warmup 3 (BENCH_ARGS= extra args)
#   prof     rocprofv3 --kernel-trace --stats of the headline command
#   proflegs the same over tools/prof_legs.py
#   pmc      PMC passes (tools/pmc.sh) of the headline workload -> pmc_traffic.json
#   pmclegs  PMC passes over tools/prof_legs.py -> pmc_legs.json
# Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-/root/repo}"
export TMPDIR=/tmp
O=gpurun_out/r04
mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "[$(date +%T)] $name"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1 || { echo "$name failed rc=$?"; tail -40 $O/$name.log; exit 1; }; }
for st in ${STAGES:-smoke tests bench}; do
  case $st in
    ab)
      for i in ${REPS:-1 2 3}; do
        for spec in ${AB:-byte:nw.nib_codes=0 nib16x10: nib8x19:nw.narrow_walk=1}; do
          tag=${spec%%:*}; opts=${spec#*:}; args=""
          for o in ${opts//,/ }; do args="$args --opt $o"; done
          step ab_${tag}_$i 120 python tools/ab_c2.py --tag $tag $args $AB_ARGS
          tail -1 $O/ab_${tag}_$i.log
        done
      done ;;
    cumap) step cumap 300 python tools/cu_map.py --out $O/cu_map.json
           tail -1 $O/cumap.log | cut -c1-1500 ;;
    pipe)
      for c in ${PIPE_CASES:-"-1" "0" "32 contiguous" "32 balanced" "64 balanced" "16 balanced" "48 balanced"}; do
        set -- $c
        step pipe_$1_${2:-x} 120 python tools/cu_pipeline.py --walk-cus $1 --layout ${2:-balanced} --map $O/cu_map.json
        tail -1 $O/pipe_$1_${2:-x}.log
      done ;;
    pipetrace) step pipetrace 300 rocprofv3 --kernel-trace -d $O/pipetrace -o run --output-format csv -- python3 tools/cu_pipeline.py ${PIPE_TRACE:---walk-cus 32 --layout balanced --steps 10 --warmup 2} --map $O/cu_map.json
               python3 tools/trace_overlap.py $O/pipetrace --out $O/pipe_overlap.json || exit 1 ;;
    rowfloor) step rowfloor 120 tools/micro/row_pk_floor 782 100000 5 1
              step rowfloor4 120 tools/micro/row_pk_floor 782 100000 5 4
              step rowfloor2 120 tools/micro/row_pk_floor 1564 50000 5 1
              step rowfloor24 120 tools/micro/row_pk_floor 1024 50000 5 4
              cat $O/rowfloor.log $O/rowfloor4.log $O/rowfloor2.log $O/rowfloor24.log ;;
    spans) step spans 600 python tools/spans_sweep.py ${SPAN_CASES:-4:1024:shared,4:1024:unique,8:1024:shared,8:1024:unique,2:1024:shared}
           cut -c1-400 $O/spans.log ;;
    abpipe)
      for i in ${REPS:-1 2 3}; do
        step abpipe_seq_$i 300 python bench.py --steps 20 --warmup 3 --legs none --no-cpu-baseline --no-pipeline
        tail -1 $O/abpipe_seq_$i.log | cut -c1-200
        step abpipe_pipe_$i 300 python bench.py --steps 20 --warmup 3 --legs none --no-cpu-baseline
        tail -1 $O/abpipe_pipe_$i.log | cut -c1-200
      done ;;
    spanq)
      GPU_MAX_HW_QUEUES=4 step spanq4 600 python tools/spans_sweep.py ${SPANQ4:-3:1024,4:1024,5:1024,6:1024,4:1024:shared:32,4:1024:shared:48}
      cut -c1-260 $O/spanq4.log
      GPU_MAX_HW_QUEUES=16 step spanq16 600 python tools/spans_sweep.py ${SPANQ16:-4:1024,8:1024}
      cut -c1-260 $O/spanq16.log ;;
    spanx)
      step spanx 900 python tools/spans_sweep.py ${SPANX:-7:1024,9:1024,10:1024,12:1024,16:1024,4:1024:reserved:62,8:1024:reserved:31}
      cut -c1-300 $O/spanx.log ;;
    spantrace)
      for n in ${SPAN_TRACE_N:-4 8}; do
        step spantrace_$n 300 rocprofv3 --kernel-trace -d $O/spantrace_$n -o run --output-format csv -- python3 tools/span_trace.py --spans $n
        python3 tools/span_trace.py --report $O/spantrace_$n --spans $n > $O/spantrace_$n.json || exit 1
        cut -c1-1500 $O/spantrace_$n.json
      done ;;
    spansolo)
      for n in ${SPAN_SOLO_N:-2 4 8}; do
        step spansolo_$n 300 python3 tools/span_trace.py --spans $n --solo
        tail -1 $O/spansolo_$n.log
      done ;;
    cuocc) step cuocc 120 python tools/cu_occupancy.py
           cat $O/cuocc.log | grep mask_cus ;;
    abwpg)
      for i in ${REPS:-1 2}; do
        for w in 1 4; do
          step abwpg_c4_${w}_$i 200 python tools/bench_long.py --len 100000 --reps 3 --opt nw.rows_wpg=$w
          echo "wpg=$w $(tail -1 $O/abwpg_c4_${w}_$i.log | cut -c1-300)"
          step abwpg_c4so_${w}_$i 200 python tools/bench_long.py --len 100000 --reps 3 --score-only --opt nw.rows_wpg=$w
          echo "wpg=$w so $(tail -1 $O/abwpg_c4so_${w}_$i.log | cut -c1-300)"
        done
      done
      for w in 1 4; do
        step abwpg_spans_$w 600 python tools/spans_sweep.py 2:1024,4:1024,8:1024 nw.rows_wpg=$w
        grep -v amdgpu.ids $O/abwpg_spans_$w.log | cut -c1-330 | sed "s/^/wpg=$w /"
      done
      step abwpg_c1 200 python tools/bench_long.py --len 1000 --reps 20
      tail -1 $O/abwpg_c1.log | cut -c1-300 ;;
    ablone)
      for i in ${REPS:-1 2}; do
        for w in 0 1; do
          step ablone_c4_${w}_$i 200 python tools/bench_long.py --len 100000 --reps 3 --opt nw.rows_lone=$w
          echo "lone=$w $(tail -1 $O/ablone_c4_${w}_$i.log | cut -c1-300)"
          step ablone_c4so_${w}_$i 200 python tools/bench_long.py --len 100000 --reps 3 --score-only --opt nw.rows_lone=$w
          echo "lone=$w so $(tail -1 $O/ablone_c4so_${w}_$i.log | cut -c1-300)"
        done
      done
      for w in 0 1; do
        step ablone_spans_$w 600 python tools/spans_sweep.py 2:1024,4:1024,8:1024 nw.rows_lone=$w
        grep -v amdgpu.ids $O/ablone_spans_$w.log | cut -c1-330 | sed "s/^/lone=$w /"
        step ablone_c1_$w 200 python tools/bench_long.py --len 1000 --reps 20 --opt nw.rows_lone=$w
        echo "lone=$w c1 $(tail -1 $O/ablone_c1_$w.log | cut -c1-300)"
      done ;;
    ablone8)
      for i in 1 2; do
        for w in 0 1; do
          step ablone8_${w}_$i 600 python tools/spans_sweep.py 8:1024,8:1024 nw.rows_lone=$w
          grep -v amdgpu.ids $O/ablone8_${w}_$i.log | python3 -c "import sys,json; [print('lone=$w', l.split()[1], json.loads(l[l.index('{'):])['fill_ms'], json.loads(l[l.index('{'):])['walk_ms']) for l in sys.stdin if '{' in l]"
        done
      done
      step spanleg 600 python bench.py --steps 2 --warmup 1 --legs c4,c4_spans --no-cpu-baseline
      tail -1 $O/spanleg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); v=d['configs']['c4_spans']; print(v['fill_ms'], v['walk_ms'])" ;;
    abbase)  # SALN_LIB=libsaln_base.so (an earlier tree) against the in-tree library
      for i in ${REPS:-1 2 3}; do
        for pp in "" "--pipeline"; do
          SALN_LIB=$PWD/sequencealigning_amd/${ABLIB:-libsaln_base.so} step abbase_b_$i 120 python tools/ab_c2.py --tag ${ABLIB:-base} $pp
          tail -1 $O/abbase_b_$i.log
          step abbase_n_$i 120 python tools/ab_c2.py --tag new $pp
          tail -1 $O/abbase_n_$i.log
        done
      done ;;
    abprof)
      step abprof_chk 200 python tools/bench_avsa.py --nq 1000 --ndb 100000 --reps 2 --check --opt nw.avsa_profile=1
      tail -1 $O/abprof_chk.log | cut -c1-400
      for i in ${REPS:-1 2}; do
        for w in 0 1; do
          step abprof_${w}_$i 200 python tools/bench_avsa.py --nq 1000 --ndb 100000 --reps 3 --opt nw.avsa_profile=$w
          echo "prof=$w $(tail -1 $O/abprof_${w}_$i.log | cut -c1-300)"
        done
      done ;;
    abg4)  # 4-row boundary groups (libsaln_g4.so) against 8 on C4 / C1 / spans
      for i in 1 2; do
        for v in g8 g4; do
          lib=""; [[ $v == g4 ]] && lib="SALN_LIB=$PWD/sequencealigning_amd/libsaln_g4.so"
          step abg4_c4_${v}_$i 200 env $lib python tools/bench_long.py --len 100000 --reps 3
          echo "$v c4 $(tail -1 $O/abg4_c4_${v}_$i.log | cut -c150-330)"
          step abg4_so_${v}_$i 200 env $lib python tools/bench_long.py --len 100000 --reps 3 --score-only
          echo "$v so $(tail -1 $O/abg4_so_${v}_$i.log | cut -c150-330)"
          step abg4_c1_${v}_$i 200 env $lib python tools/bench_long.py --len 1000 --reps 20
          echo "$v c1 $(tail -1 $O/abg4_c1_${v}_$i.log | cut -c130-300)"
        done
      done ;;
    hostt) step hostt 200 python tools/bench_host.py --reps 3 --opt host.timing=1
           grep -v amdgpu.ids $O/hostt.log | tail -24 ;;
    abwalk)  # walker variants (sequential steps: the walk's own time)
      for i in 1 2; do
        for v in base noeq new; do
          lib=""; [[ $v != new ]] && lib="SALN_LIB=$PWD/sequencealigning_amd/libsaln_$v.so"
          step abwalk_${v}_$i 120 env $lib python tools/ab_c2.py --tag $v
          tail -1 $O/abwalk_${v}_$i.log | cut -c1-220
        done
      done ;;
    abfree)  # C5 query profiles: bonuses in the extension-free frame (nw.pk_tab) against penalties
      step abfree_chk 200 python tools/bench_avsa.py --nq 1000 --ndb 100000 --reps 2 --check --opt nw.pk_tab=1
      tail -1 $O/abfree_chk.log | cut -c1-400
      for i in ${REPS:-1 2}; do
        for w in 0 1; do
          step abfree_${w}_$i 200 python tools/bench_avsa.py --nq 1000 --ndb 100000 --reps 3 --opt nw.pk_tab=$w
          echo "tab=$w $(tail -1 $O/abfree_${w}_$i.log | cut -c1-300)"
        done
      done ;;
    abmax3)  # H as one v_pk_maximum3_f16 in the extension-free frame vs two u16 maxima (libsaln_nomax3.so)
      for i in 1 2; do
        for v in nomax3 new; do
          lib=""; [[ $v != new ]] && lib="SALN_LIB=$PWD/sequencealigning_amd/libsaln_$v.so"
          step abm3_${v}_$i 120 env $lib python tools/ab_c2.py --tag $v
          tail -1 $O/abm3_${v}_$i.log | cut -c1-220
          step abm3p_${v}_$i 120 env $lib python tools/ab_c2.py --pipeline --tag $v
          tail -1 $O/abm3p_${v}_$i.log | cut -c1-220
          step abm3a_${v}_$i 200 env $lib python tools/bench_avsa.py --nq 1000 --ndb 100000 --reps 3
          echo "$v $(tail -1 $O/abm3a_${v}_$i.log | cut -c1-260)"
        done
      done ;;
    abmul)  # walker I-open gather with a 24-bit multiply (new) vs the 32-bit one (libsaln_base.so)
      for i in 1 2 3; do
        for v in base new; do
          lib=""; [[ $v != new ]] && lib="SALN_LIB=$PWD/sequencealigning_amd/libsaln_$v.so"
          step abmul_${v}_$i 120 env $lib python tools/ab_c2.py --tag $v
          tail -1 $O/abmul_${v}_$i.log | cut -c1-220
          step abmulp_${v}_$i 120 env $lib python tools/ab_c2.py --pipeline --tag $v
          tail -1 $O/abmulp_${v}_$i.log | cut -c1-220
        done
      done ;;
    abgen)  # all-vs-all classes without profiles (250 / 400 bp): table penalties (nw.pk_tab) vs xor
      for i in 1 2; do
        for L in 250 400; do
          for w in 0 1; do
            step abgen_${L}_${w}_$i 200 python tools/bench_avsa.py --nq 500 --ndb 50000 --len $L --reps 3 --opt nw.pk_tab=$w
            echo "len=$L tab=$w $(tail -1 $O/abgen_${L}_${w}_$i.log | cut -c1-240)"
          done
        done
      done ;;
    abtab)  # table-penalty fill (nw.pk_tab) against the default: sequential and pipelined steps
      for i in 1 2; do
        for w in 0 1; do
          step abtab_${w}_$i 120 python tools/ab_c2.py --tag tab$w --opt nw.pk_tab=$w
          tail -1 $O/abtab_${w}_$i.log | cut -c1-220
          step abtabp_${w}_$i 120 python tools/ab_c2.py --pipeline --tag tab$w --opt nw.pk_tab=$w
          tail -1 $O/abtabp_${w}_$i.log | cut -c1-220
        done
      done ;;
    clileg) step clileg 600 python bench.py --steps 2 --warmup 1 --legs cli
            tail -1 $O/clileg.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['configs']['cli']))" ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests) step tests 1100 python -u -m pytest ${TESTS:-tests} -m gpu -x -q --timeout 300 --timeout-method thread
           tail -3 $O/tests.log ;;
    bench) step bench 900 python bench.py --steps 20 --warmup 3 $BENCH_ARGS
           tail -1 $O/bench.log | cut -c1-1500 ;;
    prof)  step prof_c2 600 rocprofv3 --kernel-trace --stats -d $O/prof_c2 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --legs none ;;
    proflegs) step prof_legs 900 rocprofv3 --kernel-trace --stats -d $O/prof_legs -o run --output-format csv -- python3 tools/prof_legs.py --legs ${PROF_LEGS:-c1,c3,c3_affine,c4,c5} ;;
    pmc)   PMC_SETS=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU;SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU"} step pmc 900 bash tools/pmc.sh
           python3 tools/pmc_traffic.py gpurun_out/pmc $O/pmc_traffic.json r04 nw > /dev/null || exit 1 ;;
    pmclegs) PMC_SCRIPT=tools/prof_legs.py PMC_SETS=${PMC_SETS:-"FETCH_SIZE;WRITE_SIZE;SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU"} step pmc_legs 1100 bash tools/pmc.sh --legs ${PROF_LEGS:-c1,c3,c3_affine,c4,c5}
           python3 tools/pmc_traffic.py gpurun_out/pmc $O/pmc_legs.json r04 legs > /dev/null || exit 1 ;;
    *) echo "unknown stage $st"; exit 2 ;;
  esac
done
echo done
