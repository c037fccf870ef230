#!/bin/bash
# Re-test finish of the systolic fill (_lr) vs default, alternated twice on config 3, then its tests.
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
for v in "" _lr "" _lr; do
  FLEETPLACE_LIB=$root/fleetflow_amd/libfleetplace$v.so timeout -k 10 200 python -u tools/sys_sweep.py --opt link_publish \
    --values 32 --loads c3 --reps 5 >> gpurun_out/${tag}_ab$v.jsonl 2>&1 || { echo "ab $v failed"; exit 1; }
  echo "lib$v"; grep load gpurun_out/${tag}_ab$v.jsonl | tail -1 | cut -c1-120
done
FLEETPLACE_LIB=$root/fleetflow_amd/libfleetplace_lr.so timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_geometry.py tests/test_gpu_parity.py \
  -k "systolic or config3 or config2 or config5" -x -v --timeout 300 --timeout-method thread > gpurun_out/${tag}_tests_lr.log 2>&1 \
  || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests_lr.log; exit 1; }
tail -1 gpurun_out/${tag}_tests_lr.log
