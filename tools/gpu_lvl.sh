#!/bin/bash
# Levelizer timing on the GPU box: config 5 with the in-tree pre-pass on and off, and a
# rocprofv3 kernel-stats pass of the default.   tools/gpu_lvl.sh <tag>
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/lvl_time.py tree_jump=0 > gpurun_out/${tag}_lvl_tree0.txt 2>&1 || { tail -20 gpurun_out/${tag}_lvl_tree0.txt; exit 1; }
timeout -k 10 120 python -u tools/lvl_time.py > gpurun_out/${tag}_lvl_tree1.txt 2>&1 || { tail -20 gpurun_out/${tag}_lvl_tree1.txt; exit 1; }
cat gpurun_out/${tag}_lvl_tree0.txt gpurun_out/${tag}_lvl_tree1.txt | grep ms_per_step
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d "$root/gpurun_out/${tag}_lvlprof" -o run -- python3 "$root/tools/lvl_time.py" \
  > gpurun_out/${tag}_lvlprof.log 2>&1 || { tail -20 gpurun_out/${tag}_lvlprof.log; exit 1; }
f=$(find "$root/gpurun_out/${tag}_lvlprof" -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/${tag}_lvl_kernel_stats.csv && cut -d, -f1-4 gpurun_out/${tag}_lvl_kernel_stats.csv | head -25
