#!/bin/bash
# 512 scenarios per GPU (the N = 8 per-rank load): narrow geometries with / without the systolic fill
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
: > gpurun_out/${tag}_geo512.jsonl
for g in "" "pipe_w=3,pipe_seg=12" "pipe_w=2,pipe_seg=8" "pipe_w=4,pipe_seg=8" "pipe_w=4,pipe_seg=4"; do
  timeout -k 10 200 python -u tools/sys_sweep.py --set "$g" --opt systolic --values 0,32 --loads c4x512 --reps 3 \
    >> gpurun_out/${tag}_geo512.jsonl 2>&1 || { echo "geo $g failed"; tail -5 gpurun_out/${tag}_geo512.jsonl; exit 1; }
done
grep load gpurun_out/${tag}_geo512.jsonl | cut -c1-330
timeout -k 10 400 python -u tools/pipe_model.py gpurun_out/${tag}_pipe_model.json > gpurun_out/${tag}_pipe_model.log 2>&1 || { echo "model failed"; tail gpurun_out/${tag}_pipe_model.log; exit 1; }
tail -2 gpurun_out/${tag}_pipe_model.log | cut -c1-300
