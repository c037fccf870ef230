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
