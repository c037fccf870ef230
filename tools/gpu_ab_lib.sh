#!/bin/bash
# A/B of library builds (tools/build_variant.sh) on device-resident loads: FFD kernel ms per load
#   tools/gpu_ab_lib.sh <tag> "<suffix> ..." [loads]   ("-" = the default build)
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}; libs=${2:-"-"}; loads=${3:-c4x4096,c3}
mkdir -p gpurun_out
for v in $libs; do
  [ "$v" = "-" ] && v=""
  FLEETPLACE_LIB=$root/fleetflow_amd/libfleetplace$v.so timeout -k 10 300 python -u tools/sys_sweep.py --opt link_publish \
    --values 32 --loads $loads --reps 3 > gpurun_out/${tag}_ab$v.jsonl 2>&1 || { echo "ab $v failed"; tail gpurun_out/${tag}_ab$v.jsonl; exit 1; }
  echo "lib$v"; cut -c1-160 gpurun_out/${tag}_ab$v.jsonl
done
