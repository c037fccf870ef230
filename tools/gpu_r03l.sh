#!/bin/bash
# bench vs sweep on one box: the config-4 FFD kernel at 4096 and 512 scenarios
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/sys_sweep.py --opt link_publish --values 32 --loads c4x4096,c4x512 --reps 3 > gpurun_out/${tag}_sweep.jsonl 2>&1 || exit 1
cut -c1-120 gpurun_out/${tag}_sweep.jsonl
for sc in 4096 512; do
  timeout -k 10 200 python -u bench.py --scenarios $sc --no-legs --no-stage2 --no-cpu-baseline --steps 10 > gpurun_out/${tag}_b$sc.json 2> gpurun_out/${tag}_b$sc.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/${tag}_b$sc.json'));print($sc, round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3))"
done
timeout -k 10 200 python -u tools/stream_ab.py 512 > gpurun_out/${tag}_stream512.jsonl 2>&1 || exit 1
cat gpurun_out/${tag}_stream512.jsonl
