#!/bin/bash
# A/B on the GPU box: bench (kernel ms, step ms) of each library variant, then the stats timeline of
# each stats variant.  tools/ab.sh "<suffix> ..." "<stats suffix> ..."   ("-" = default build)
set -e
for v in $1; do
  [ "$v" = "-" ] && v=""
  FLEETPLACE_LIB=$PWD/fleetflow_amd/libfleetplace$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 5 --warmup 1 > gpurun_out/ab$v.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/ab$v.json'));print('lib$v', round(d['roofline']['kernel_ms'],3), round(d['ms_per_step'],3))"
done
for v in $2; do
  [ "$v" = "-" ] && v=""
  FLEETPLACE_LIB=$PWD/fleetflow_amd/libfleetplace_stats$v.so TIMELINE=gpurun_out/tl$v.csv timeout -k 10 120 python tools/pipe_stats.py > gpurun_out/ps$v.txt 2>&1
done
