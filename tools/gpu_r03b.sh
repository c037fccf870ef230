#!/bin/bash
# ubench (systolic variants) + gpu_r03.sh
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}; shift
mkdir -p gpurun_out
timeout -k 10 120 ./tools/ubench/systolic_v > gpurun_out/${tag}_systolic_v.txt 2>&1 || { echo "ubench failed"; tail gpurun_out/${tag}_systolic_v.txt; exit 1; }
bash tools/gpu_r03.sh $tag "$@"
