#!/bin/bash
# Levelizer counting-sort check: levelizer parity tests, then config-5 levelize time with the
# counting sort and with rocprim's radix sort (level_sort=0) in one call, then the trace.
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_consumers.py tests/test_gpu_errors.py -k "lev or config5 or waves or corrupt or nothing" -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_tests.log
timeout -k 10 200 python -u tools/lvl_time.py > gpurun_out/${tag}_lvl.jsonl 2>&1 || { echo "lvl failed"; tail gpurun_out/${tag}_lvl.jsonl; exit 1; }
echo "counting sort"; cat gpurun_out/${tag}_lvl.jsonl
timeout -k 10 200 python -u tools/lvl_time.py level_sort=0 > gpurun_out/${tag}_lvl_radix.jsonl 2>&1 || { echo "lvl radix failed"; tail gpurun_out/${tag}_lvl_radix.jsonl; exit 1; }
echo "radix sort"; cat gpurun_out/${tag}_lvl_radix.jsonl
timeout -k 10 300 python -u tools/lvl_time.py > gpurun_out/${tag}_lvl2.jsonl 2>&1 || exit 1
echo "counting sort again"; cat gpurun_out/${tag}_lvl2.jsonl
bash tools/gpu_r03t.sh
