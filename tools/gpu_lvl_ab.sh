#!/bin/bash
# A/B of levelizer builds on config 5:  tools/gpu_lvl_ab.sh <tag> "<suffix> ..."   ("-" = default)
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}; libs=${2:-"-"}
mkdir -p gpurun_out
for rep in 1 2; do
for v in $libs; do
  [ "$v" = "-" ] && v=""
  FLEETPLACE_LIB=$root/fleetflow_amd/libfleetplace$v.so timeout -k 10 120 python -u tools/lvl_time.py \
    > gpurun_out/${tag}_lvl${v}_$rep.txt 2>&1 || { echo "lvl $v failed"; tail gpurun_out/${tag}_lvl${v}_$rep.txt; exit 1; }
  echo "lib$v rep $rep $(grep ms_per gpurun_out/${tag}_lvl${v}_$rep.txt | tail -1)"
done
done
