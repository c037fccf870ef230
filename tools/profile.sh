#!/bin/bash
# rocprofv3 evidence for the bench workload (run on the GPU box via gpurun):
#   1. kernel trace + stats  2. FETCH_SIZE pass  3. WRITE_SIZE pass (separate: TCC slots)
# Both bench legs (config 4 at 4096 scenarios, config 3) run in every pass.
# Usage: tools/profile.sh <tag>   -> gpurun_out/prof_<tag>/{trace,fetch,write}
set -eo pipefail
tag=${1:-r02}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/prof_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
args="$root/bench.py --no-cpu-baseline --steps 2 --warmup 1 --config3-steps 1"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- python3 $args > "$out/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- python3 $args > "$out/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- python3 $args > "$out/write.log" 2>&1
echo "profile $tag done"
