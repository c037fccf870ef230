#!/bin/bash
# Prescan skip (default build) and the todo-skip variant: A/B, then the config-4 / geometry parity tests.
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
bash tools/gpu_ab_lib.sh $tag "- _ts -" c4x4096,c4x512 || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_geometry.py tests/test_gpu_links.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
