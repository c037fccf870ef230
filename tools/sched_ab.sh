#!/bin/bash
# Scheduler-strategy A/B of the non-FFD kernels (tools/sched_ab.sh <tag>): the sort path and the
# stage-2 sweep from bench.py's config-4 + stage-2 legs, the levelizer from tools/lvl_time.py,
# each library build twice.  Variant builds: fleetflow_amd/libfleetplace_<file>_<strategy>.so.
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
for rep in 1 2; do
  for v in "" _place_imo _place_iilp _feas_imo _feas_iilp; do
    FLEETPLACE_LIB=$root/fleetflow_amd/libfleetplace$v.so timeout -k 10 200 python -u bench.py --no-legs --no-cpu-baseline \
      --steps 5 > gpurun_out/${tag}_bench${v}_${rep}.json 2> gpurun_out/${tag}_bench${v}_${rep}.err || { echo "bench $v failed"; tail gpurun_out/${tag}_bench${v}_${rep}.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'rep', sys.argv[3], 'step', round(d['ms_per_step'],3), d['breakdown_ms'], 'stage2', round(d['stage2']['kernel_ms'],3))" gpurun_out/${tag}_bench${v}_${rep}.json "lib$v" $rep
  done
  for v in "" _order_imo _order_iilp; do
    FLEETPLACE_LIB=$root/fleetflow_amd/libfleetplace$v.so timeout -k 10 120 python -u tools/lvl_time.py > gpurun_out/${tag}_lvl${v}_${rep}.txt 2>&1 || { echo "lvl $v failed"; tail gpurun_out/${tag}_lvl${v}_${rep}.txt; exit 1; }
    echo "lib$v rep $rep"; grep ms_per_step gpurun_out/${tag}_lvl${v}_${rep}.txt
  done
done
