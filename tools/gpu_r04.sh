#!/bin/bash
# Round-4 GPU session steps (run on the box via gpurun from the repo root):
#   tools/gpu_r04.sh <tag> <step>...   steps: ubench | tests:<pytest -k expr> | alltests | sweep:<opt>:<values>:<loads> | sortstats | pipestats | bench
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}; shift
mkdir -p gpurun_out
for step in "$@"; do
  case "$step" in
    ubench)
      (cd tools/ubench && timeout -k 10 60 ./lat_salu && timeout -k 10 60 ./resolve) > gpurun_out/${tag}_ubench.txt 2>&1 \
        || { echo "ubench failed"; tail -20 gpurun_out/${tag}_ubench.txt; exit 1; } ;;
    tests:*)
      k=${step#tests:}
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$k" \
        > gpurun_out/${tag}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${tag}_tests.log; exit 1; } ;;
    alltests)
      timeout -k 10 1100 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
        > gpurun_out/${tag}_alltests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${tag}_alltests.log; exit 1; } ;;
    sweep:*)
      IFS=: read -r _ opt vals loads <<< "$step"
      timeout -k 10 400 python -u tools/sys_sweep.py --opt "$opt" --values "$vals" --loads "$loads" --reps 3 \
        > gpurun_out/${tag}_sweep_${opt}.jsonl 2>&1 || { echo "sweep failed"; tail -20 gpurun_out/${tag}_sweep_${opt}.jsonl; exit 1; }
      cut -c1-200 gpurun_out/${tag}_sweep_${opt}.jsonl ;;
    pipestats)
      FLEETPLACE_LIB=$PWD/fleetflow_amd/libfleetplace_stats.so timeout -k 10 200 python -u tools/pipe_stats.py 4096 \
        > gpurun_out/${tag}_pipestats_c4.txt 2>&1 || { echo "pipestats failed"; tail -20 gpurun_out/${tag}_pipestats_c4.txt; exit 1; }
      cat gpurun_out/${tag}_pipestats_c4.txt ;;
    sortstats)
      timeout -k 10 300 python -u tools/sort_stats.py > gpurun_out/${tag}_sortstats.txt 2>&1 \
        || { echo "sortstats failed"; tail -20 gpurun_out/${tag}_sortstats.txt; exit 1; }
      cat gpurun_out/${tag}_sortstats.txt ;;
    bench)
      timeout -k 10 600 python -u bench.py > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err \
        || { echo "bench failed"; tail -30 gpurun_out/${tag}_bench.err; exit 1; } ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
  echo "step $step ok"
done
