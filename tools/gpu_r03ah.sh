#!/bin/bash
# Systolic-call statistics on config 3 (stats builds with / without the staircase live filter), then
# the FFD A/B of the staircase filter on configs 3 and 2.
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
for v in _stats _stats_st; do
  FLEETPLACE_LIB=$root/fleetflow_amd/libfleetplace$v.so timeout -k 10 300 python -u tools/sys_stats.py > gpurun_out/${tag}_sys$v.json 2>&1 \
    || { echo "sys stats $v failed"; tail gpurun_out/${tag}_sys$v.json; exit 1; }
  echo "$v"; grep calls gpurun_out/${tag}_sys$v.json
done
bash tools/gpu_ab_lib.sh $tag "- _st -" c3,c2 || exit 1
# value-bitmap load unroll: config-4 step and sort time, old build (_bm0) vs default
for v in _bm0 "" _bm0 ""; do
  FLEETPLACE_LIB=$root/fleetflow_amd/libfleetplace$v.so timeout -k 10 200 python -u bench.py --no-legs --no-stage2 --no-cpu-baseline --steps 10 \
    > gpurun_out/${tag}_bm$v.json 2> gpurun_out/${tag}_bm$v.err || { echo "bench $v failed"; tail gpurun_out/${tag}_bm$v.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['ms_per_step'], d['breakdown_ms'])" gpurun_out/${tag}_bm$v.json "lib$v"
done
