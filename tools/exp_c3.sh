# geometry sweep for the single-scenario configs: bash tools/exp_c3.sh <config> "W SEG" ...
c=$1; shift
for cfg in "$@"; do
  set -- $cfg
  FLEETPLACE_PIPE_W=$1 FLEETPLACE_PIPE_SEG=$2 timeout -k 10 200 python tools/bench_configs.py --only $c --no-cpu --reps 3 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('cfg $c W=$1 SEG=$2', round(d['gpu_wall_ms'],3), round(d['ffd_kernel_ms'],3), d['bit_exact'])" || echo "W=$1 SEG=$2 failed"
done
