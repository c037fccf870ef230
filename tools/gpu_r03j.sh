#!/bin/bash
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/stream_ab.py 4096 > gpurun_out/${tag}_stream_ab.jsonl 2>&1 || { echo "stream_ab failed"; tail gpurun_out/${tag}_stream_ab.jsonl; exit 1; }
cat gpurun_out/${tag}_stream_ab.jsonl
bash tools/gpu_r03c.sh $tag
