#!/bin/bash
# Levelizer timing on the GPU box: config 5 (bench.py's levelize leg) and a rocprofv3
# kernel-stats pass of it.   tools/gpu_lvl.sh <tag> [option=value ...]
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
mkdir -p gpurun_out
tag=${1:?tag}; shift
timeout -k 10 120 python -u tools/lvl_time.py "$@" > gpurun_out/${tag}_lvl.txt 2>&1 || { tail -20 gpurun_out/${tag}_lvl.txt; exit 1; }
grep ms_per_step gpurun_out/${tag}_lvl.txt
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/gpurun_out/${tag}_lvlprof" -o run -- python3 "$root/tools/lvl_time.py" "$@" \
  > gpurun_out/${tag}_lvlprof.log 2>&1 || { tail -20 gpurun_out/${tag}_lvlprof.log; exit 1; }
f=$(find "$root/gpurun_out/${tag}_lvlprof" -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/${tag}_lvl_kernel_stats.csv && cut -d, -f1-4 gpurun_out/${tag}_lvl_kernel_stats.csv | head -25
