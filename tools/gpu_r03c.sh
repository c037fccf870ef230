#!/bin/bash
# Diagnostics build counters (configs 4 / 512 / 3) + SQ counter passes over the config-4 bench.
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
bash tools/gpu_diag.sh $tag || exit 1
timeout -k 10 600 bash tools/pmc_sq.sh $tag || { echo "sq failed"; exit 1; }
echo "gpu_r03c $tag done"
