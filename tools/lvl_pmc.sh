#!/bin/bash
# HBM bytes of config 5's levelization (rocprofv3 PMC, one counter per pass: FETCH_SIZE, then
# WRITE_SIZE) on the GPU box:  tools/lvl_pmc.sh <tag>  -> gpurun_out/lvlpmc_<tag>/{fetch,write}
# Summarise on the CPU side with tools/summarize_lvl_pmc.py <tag>.
set -eo pipefail
tag=${1:?tag}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/lvlpmc_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- python3 "$root/tools/lvl_time.py" > "$out/fetch.log" 2>&1
timeout -k 10 180 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- python3 "$root/tools/lvl_time.py" > "$out/write.log" 2>&1
echo "lvl pmc $tag done"
