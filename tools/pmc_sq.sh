#!/bin/bash
# SQ/SQC counter passes over the bench workload (one rocprofv3 run per pass).
# Usage: tools/pmc_sq.sh <tag>  -> gpurun_out/sq_<tag>/p<i>   (env: FLEETPLACE_LIB selects a library
# build, SQ_PASSES the passes to run, default "1 2 3")
set -eo pipefail
tag=${1:-r01}
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/sq_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
args="$root/bench.py --no-cpu-baseline --no-legs --no-stage2 --steps 2 --warmup 1"
passes=("SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
        "SQ_WAIT_ANY SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS SQ_IFETCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS"
        "SQ_INSTS_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES")
for i in ${SQ_PASSES:-1 2 3}; do
  pmc=${passes[$((i-1))]}
  timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d "$out/p$i" -o run -- python3 $args > "$out/p$i.log" 2>&1
done
echo "sq $tag done"
