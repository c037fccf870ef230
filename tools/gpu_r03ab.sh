#!/bin/bash
# todo skip on by default: A/B against the build without it (config 4 and 3), then the -m gpu suite.
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
bash tools/gpu_ab_lib.sh $tag "- _nts" c4x4096,c3 || exit 1
bash tools/gpu_round.sh $tag tests || exit 1
