#!/bin/bash
# r04j: config-4 kernel traces of HEAD and of the r04c build (non-FFD regression hunt), and the
# levelizer timing after the atomics fix.
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tools/ktrace.sh r04j_head > gpurun_out/r04j_kt_head.txt 2>&1 || { cat gpurun_out/r04j_kt_head.txt; exit 1; }
cat gpurun_out/r04j_kt_head.txt
FLEETPLACE_LIB=$root/fleetflow_amd/libfleetplace_r04c.so tools/ktrace.sh r04j_r04c > gpurun_out/r04j_kt_r04c.txt 2>&1 || { cat gpurun_out/r04j_kt_r04c.txt; exit 1; }
cat gpurun_out/r04j_kt_r04c.txt
tools/gpu_lvl.sh r04j
