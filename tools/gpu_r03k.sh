#!/bin/bash
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_consumers.py -k "lev or config5 or waves" -x -v --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${tag}_tests.log; exit 1; }
tail -2 gpurun_out/${tag}_tests.log
timeout -k 10 200 python -u tools/lvl_time.py > gpurun_out/${tag}_lvl.jsonl 2>&1 || { echo "lvl failed"; tail gpurun_out/${tag}_lvl.jsonl; exit 1; }
cat gpurun_out/${tag}_lvl.jsonl
bash tools/gpu_round.sh $tag scale && for sc in 2048 1024 512; do python3 -c "import json;d=json.load(open('gpurun_out/${tag}_scale_$sc.json'));print($sc, round(d['ms_per_step'],3), round(d['roofline']['kernel_ms'],3), round(d['breakdown_ms']['sort'],3))"; done
timeout -k 10 300 python -u -m pytest tests/test_gpu_scen_sort.py -x -q --timeout 200 --timeout-method thread \
  > gpurun_out/${tag}_scen_tests.log 2>&1 || { echo "scen tests failed"; tail -30 gpurun_out/${tag}_scen_tests.log; exit 1; }
tail -1 gpurun_out/${tag}_scen_tests.log
timeout -k 10 300 python -u tools/sys_sweep.py --opt payload_lds --values 1,2,1,2 --loads c4x4096 --reps 3 > gpurun_out/${tag}_payload.jsonl 2>&1 || exit 1
cat gpurun_out/${tag}_payload.jsonl | cut -c1-140
