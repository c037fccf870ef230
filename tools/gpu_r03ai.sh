#!/bin/bash
# Systolic fill: serial finish with the re-test (_lr), + stop at the first miss (_me), stop only (_meo):
# FFD A/B on configs 3 and 2, then the systolic / config-3 parity tests on _me.
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
bash tools/gpu_ab_lib.sh $tag "- _lr _me _meo -" c3,c2 || exit 1
FLEETPLACE_LIB=$root/fleetflow_amd/libfleetplace_me.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_geometry.py tests/test_gpu_parity.py \
  -k "systolic or config3 or config2" -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests_me.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests_me.log; exit 1; }
tail -1 gpurun_out/${tag}_tests_me.log
bash tools/gpu_round.sh $tag tests || exit 1
