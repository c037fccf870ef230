#!/bin/bash
# Round-3 GPU session: gpu_round (errors tests bench prof) + FETCH/WRITE calibration kernels.
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}; shift
bash tools/gpu_round.sh $tag ${*:-errors tests bench prof} || exit 1
timeout -k 10 300 bash tools/fetchcal.sh || { echo "fetchcal failed"; exit 1; }
echo "gpu_r03 $tag done"
