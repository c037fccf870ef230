#!/bin/bash
# A/B of library builds on device-resident loads (FFD kernel ms, same plan check):
#   tools/ab_variants.sh <tag> "<suffix> ..." <loads>   ("-" = the default build)
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}; libs=${2:-"-"}; loads=${3:-c4x4096,c3}
mkdir -p gpurun_out
for rep in 1 2; do
for v in $libs; do
  [ "$v" = "-" ] && v=""
  FLEETPLACE_LIB=$root/fleetflow_amd/libfleetplace$v.so timeout -k 10 300 python -u tools/sys_sweep.py --opt link_publish \
    --values 32 --loads $loads --reps 3 > gpurun_out/${tag}_ab${v}_$rep.jsonl 2>&1 || { echo "ab $v failed"; tail gpurun_out/${tag}_ab${v}_$rep.jsonl; exit 1; }
  echo "lib$v rep $rep"; grep load gpurun_out/${tag}_ab${v}_$rep.jsonl | cut -c1-120
done
done
