#!/bin/bash
# Segment width after the pass-through skips: pipe_seg 12 / 16 / 20 (default build: 16+ groups at
# three waves per SIMD; _ww4: four).
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
for v in "" _ww4; do
  FLEETPLACE_LIB=$root/fleetflow_amd/libfleetplace$v.so timeout -k 10 300 python -u tools/sys_sweep.py --opt pipe_seg \
    --values 12,16,20,12 --loads c4x4096 --reps 3 > gpurun_out/${tag}_seg$v.jsonl 2>&1 || { echo "sweep $v failed"; tail gpurun_out/${tag}_seg$v.jsonl; exit 1; }
  echo "lib$v"; cut -c1-230 gpurun_out/${tag}_seg$v.jsonl
done
