#!/bin/bash
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 400 python -u tools/sys_sweep.py --opt link_publish --values 1,8,32,64,1 --loads c4x4096 --reps 3 > gpurun_out/${tag}_publish.jsonl 2>&1 || exit 1
cut -c1-130 gpurun_out/${tag}_publish.jsonl
timeout -k 10 400 python -u tools/sys_sweep.py --opt systolic --values 0,32,0,32 --loads c3,c2 --reps 2 > gpurun_out/${tag}_systolic.jsonl 2>&1 || exit 1
cut -c1-130 gpurun_out/${tag}_systolic.jsonl
bash tools/gpu_ab_lib.sh ${tag} "- _pfm0 _pfm4 _pfm32 -" c4x4096,c3
