set -e
for W in 4 2 1 8; do
  FLEETPLACE_PIPE_W=$W timeout -k 10 120 python tools/bench_configs.py --only 2 --no-cpu --reps 5 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.readline()); print('W=$W', round(d['gpu_wall_ms'],3), round(d['ffd_kernel_ms'],3), d['bit_exact'])"
done
