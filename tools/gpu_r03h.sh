#!/bin/bash
# link publish batching: parity tests of the geometry file, then the A/B sweep
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_geometry.py tests/test_gpu_links.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 400 python -u tools/sys_sweep.py --opt link_publish --values 1,8,64,1024 --loads c4x4096,c4x512,c3 --reps 3 \
  > gpurun_out/${tag}_publish.jsonl 2>&1 || { echo "sweep failed"; tail gpurun_out/${tag}_publish.jsonl; exit 1; }
cat gpurun_out/${tag}_publish.jsonl
