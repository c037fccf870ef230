# A/B of library builds on the bench workload: tools/exp_lib.sh <suffix>...  ("" = default build)
set -e
for v in "$@"; do
  [ "$v" = "-" ] && v=""
  FLEETPLACE_LIB=$PWD/fleetflow_amd/libfleetplace$v.so timeout -k 10 120 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/exp_lib$v.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/exp_lib$v.json'));print('lib$v', d['roofline']['kernel_ms'], d['ms_per_step'])"
done
