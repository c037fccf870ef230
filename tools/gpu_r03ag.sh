#!/bin/bash
# After the pass-through skips: strong-scaling per-rank loads and the diagnostics-build latency model.
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
bash tools/gpu_round.sh $tag scale || exit 1
for sc in 2048 1024 512; do python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[1], d['ms_per_step'], d['breakdown_ms'])" gpurun_out/${tag}_scale_$sc.json; done
timeout -k 10 400 python -u tools/pipe_model.py gpurun_out/${tag}_pipe_model.json > gpurun_out/${tag}_pipe_model.log 2>&1 || { echo "model failed"; tail gpurun_out/${tag}_pipe_model.log; exit 1; }
tail -2 gpurun_out/${tag}_pipe_model.log | cut -c1-400
