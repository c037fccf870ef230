#!/bin/bash
# Diagnostics build runs (libfleetplace_stats.so): per-stage counters of config 4 (4096 and 512
# scenarios) and config 3 (spans of every global stage).  -> gpurun_out/<tag>_diag_*.txt
set -o pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
cd "$root" || exit 1
tag=${1:?tag}
timeout -k 10 200 python -u tools/pipe_stats.py 4096 > gpurun_out/${tag}_diag_c4.txt 2>&1 || { echo "c4 failed"; tail gpurun_out/${tag}_diag_c4.txt; exit 1; }
timeout -k 10 200 python -u tools/pipe_stats.py 512 > gpurun_out/${tag}_diag_c4x512.txt 2>&1 || { echo "c4x512 failed"; exit 1; }
SEED=0x5EED0003 C=1000000 N=100000 SPAN=gpurun_out/${tag}_c3_span.csv timeout -k 10 300 python -u tools/pipe_stats.py 1 \
  > gpurun_out/${tag}_diag_c3.txt 2>&1 || { echo "c3 failed"; tail gpurun_out/${tag}_diag_c3.txt; exit 1; }
cat gpurun_out/${tag}_diag_*.txt
