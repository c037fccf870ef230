#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration runs (tools/ubench/fetchcal.hip), one process and one
# counter per rocprofv3 pass (GPU box, via gpurun).  Summarise with tools/fetchcal_summary.py.
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/fetchcal
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
for k in r4 r16 g4 w4 w1 w16; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 60 rocprofv3 --pmc $ctr --output-format csv -d "$out/${k}_$ctr" -o run -- "$root/tools/ubench/fetchcal" $k \
      > "$out/${k}_$ctr.log" 2>&1
  done
done
echo "fetchcal done"
