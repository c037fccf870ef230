#!/bin/bash
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
bash tools/gpu_ab_lib.sh r03i "- _pf _pfm0 _pfm8" c4x4096,c3 || exit 1
bash tools/gpu_round.sh r03i tests bench prof
