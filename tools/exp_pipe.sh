# tuning sweep of the pipeline geometry (FLEETPLACE_PIPE_W / FLEETPLACE_PIPE_SEG), run on the GPU box
set -e
for cfg in ${CFGS:-"8 0" "4 40" "4 20" "1 10" "3 30" "5 40"}; do
  set -- $cfg
  FLEETPLACE_PIPE_W=$1 FLEETPLACE_PIPE_SEG=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/exp_$1_$2.json 2>/dev/null
  python -c "import json;d=json.load(open('gpurun_out/exp_$1_$2.json'));print('W=$1 SEG=$2', d['roofline']['kernel_ms'], d['ms_per_step'])"
done
