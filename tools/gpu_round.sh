#!/bin/bash
# One GPU session: error-path tests (isolated, short limit), the -m gpu suite, the bench
# (config 4 at 4096 + config 3 leg + CPU baseline), then the rocprofv3 passes.
# Usage: tools/gpu_round.sh <tag> [steps...]
#   steps: errors tests bench scale prof kt lvl sortstats pipestats model front ab sq sweep (default: errors tests bench prof)
#   kt = config-4 kernel trace (tools/ktrace.sh), lvl = config-5 levelizer timing + kernel stats
#   (tools/gpu_lvl.sh), sortstats / pipestats / model = diagnostics-build runs (k_scen_sort phases,
#   per-stage pipeline counters at 4096 scenarios, the latency model of tools/pipe_model.py)
set -o pipefail
tag=${1:?tag}; shift
steps=${*:-errors tests bench prof}
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
mkdir -p gpurun_out
log=gpurun_out/${tag}
for s in $steps; do
  case $s in
    errors)
      timeout -k 10 150 python -u -m pytest tests/test_gpu_errors.py -x -v --timeout 120 --timeout-method thread \
        > ${log}_errors.log 2>&1 || { echo "errors step failed"; tail -30 ${log}_errors.log; exit 1; } ;;
    tests)
      timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread \
        > ${log}_tests.log 2>&1 || { echo "tests step failed"; tail -40 ${log}_tests.log; exit 1; }
      tail -3 ${log}_tests.log ;;
    bench)
      timeout -k 10 400 python -u bench.py > ${log}_bench.json 2> ${log}_bench.err \
        || { echo "bench failed"; tail -30 ${log}_bench.err; exit 1; }
      cat ${log}_bench.json ;;
    scale)
      # per-rank loads of the strong-scaled config 4 (4096 / N scenarios on one GPU)
      for sc in 2048 1024 512; do
        timeout -k 10 200 python -u bench.py --scenarios $sc --no-legs --no-stage2 --no-cpu-baseline --steps 10 \
          > ${log}_scale_$sc.json 2> ${log}_scale_$sc.err || { echo "scale $sc failed"; tail -20 ${log}_scale_$sc.err; exit 1; }
      done ;;
    prof)
      timeout -k 10 1000 bash tools/profile.sh $tag || { echo "profile failed"; exit 1; } ;;
    kt)
      tools/ktrace.sh $tag > ${log}_kt.txt 2>&1 || { echo "kt failed"; tail -20 ${log}_kt.txt; exit 1; }
      cat ${log}_kt.txt ;;
    lvl)
      tools/gpu_lvl.sh $tag || { echo "lvl failed"; exit 1; } ;;
    sortstats)
      timeout -k 10 300 python -u tools/sort_stats.py > ${log}_sortstats.txt 2>&1 || { echo "sortstats failed"; tail ${log}_sortstats.txt; exit 1; }
      cat ${log}_sortstats.txt ;;
    pipestats|stats)
      timeout -k 10 300 python -u tools/pipe_stats.py 4096 > ${log}_pipestats.txt 2>&1 || { echo "pipestats failed"; tail ${log}_pipestats.txt; exit 1; }
      cat ${log}_pipestats.txt ;;
    model)
      timeout -k 10 400 python -u tools/pipe_model.py ${log}_pipe_model.json > ${log}_pipe_model.log 2>&1 || { echo "model failed"; tail ${log}_pipe_model.log; exit 1; } ;;
    front)
      # where a placement's cycles go at the front (diagnostics build timeline, tools/front_breakdown.py):
      # config 3 and the 512-scenario per-rank load
      SEED=0x5EED0003 C=1000000 N=100000 TIMELINE=${log}_tl_c3.csv timeout -k 10 300 python -u tools/pipe_stats.py 1 \
        > ${log}_front_c3.txt 2>&1 || { echo "front c3 failed"; tail ${log}_front_c3.txt; exit 1; }
      TIMELINE=${log}_tl_512.csv timeout -k 10 300 python -u tools/pipe_stats.py 512 \
        > ${log}_front_512.txt 2>&1 || { echo "front 512 failed"; tail ${log}_front_512.txt; exit 1; }
      python tools/front_breakdown.py ${log}_tl_c3.csv >> ${log}_front_c3.txt
      python tools/front_breakdown.py ${log}_tl_512.csv >> ${log}_front_512.txt
      tail -25 ${log}_front_c3.txt; tail -25 ${log}_front_512.txt ;;
    tl4096)
      # config 4's per-batch timeline (diagnostics build; scenario 0's segments = global stages 0-6)
      TIMELINE=${log}_tl_4096.csv timeout -k 10 300 python -u tools/pipe_stats.py 4096 \
        > ${log}_tl4096.txt 2>&1 || { echo "tl4096 failed"; tail ${log}_tl4096.txt; exit 1; }
      python tools/front_breakdown.py ${log}_tl_4096.csv 2.4 0 >> ${log}_tl4096.txt
      tail -30 ${log}_tl4096.txt ;;
    ab)
      # library variants on device-resident loads: AB_LIBS="- _suffix ...", AB_LOADS=c4x4096,c3,...
      tools/ab_variants.sh $tag "${AB_LIBS:--}" ${AB_LOADS:-c4x4096,c3} > ${log}_ab.txt 2>&1 \
        || { echo "ab failed"; tail -20 ${log}_ab.txt; exit 1; }
      cat ${log}_ab.txt ;;
    sq)
      # SQ instruction / wave counters of the config-4 kernel for each library build: SQ_LIBS="- _suffix ..."
      for v in ${SQ_LIBS:--}; do
        [ "$v" = "-" ] && v=""
        FLEETPLACE_LIB=$root/fleetflow_amd/libfleetplace$v.so SQ_PASSES=${SQ_PASSES:-1} bash tools/pmc_sq.sh ${tag}$v \
          || { echo "sq $v failed"; exit 1; }
        python tools/sq_summary.py ${tag}$v k_ffd_pipe
      done ;;
    sweep)
      # one context option over device-resident loads: SWEEP_OPT, SWEEP_VALUES, SWEEP_LOADS (tools/sys_sweep.py)
      sw=${log}_sweep_${SWEEP_OPT}${SWEEP_SET:+_$(echo $SWEEP_SET | tr ',=' '__')}.jsonl
      timeout -k 10 400 python -u tools/sys_sweep.py --opt ${SWEEP_OPT:?} --values=${SWEEP_VALUES:?} \
        --loads ${SWEEP_LOADS:-c4x512,c3} --reps 3 ${SWEEP_SET:+--set $SWEEP_SET} > $sw 2>&1 \
        || { echo "sweep failed"; tail -20 $sw; exit 1; }
      cut -c1-200 $sw | grep load ;;
    ubench)
      # one-wave group-loop microbenchmark (tools/ubench/systolic.hip, built on the CPU side)
      timeout -k 10 120 tools/ubench/systolic > ${log}_ubench.txt 2>&1 || { echo "ubench failed"; tail ${log}_ubench.txt; exit 1; }
      cat ${log}_ubench.txt ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
echo "gpu_round $tag done: $steps"
