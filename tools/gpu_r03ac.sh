#!/bin/bash
# deferred req/conf loads (default) vs FP_DEFER_RC=0: A/B, then the -m gpu suite.
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
bash tools/gpu_ab_lib.sh $tag "- _ndr -" c4x4096,c4x512 || exit 1
bash tools/gpu_round.sh $tag tests || exit 1
