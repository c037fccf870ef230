#!/bin/bash
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
bash tools/gpu_round.sh $tag errors tests || exit 1
timeout -k 10 400 python -u tools/pipe_model.py gpurun_out/${tag}_pipe_model.json > gpurun_out/${tag}_pipe_model.log 2>&1 || { echo "model failed"; tail gpurun_out/${tag}_pipe_model.log; exit 1; }
timeout -k 10 300 python -u tools/pipe_stats.py 4096 > gpurun_out/${tag}_diag_c4.txt 2>&1 || exit 1
bash tools/gpu_round.sh $tag bench prof
