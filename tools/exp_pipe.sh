# tuning sweep of the pipeline geometry (FLEETPLACE_PIPE_W / FLEETPLACE_PIPE_SEG), run on the GPU box
# usage: bash tools/exp_pipe.sh "W SEG" ...
for cfg in "$@"; do
  set -- $cfg
  FLEETPLACE_PIPE_W=$1 FLEETPLACE_PIPE_SEG=$2 timeout -k 10 120 python bench.py --no-cpu-baseline --steps 3 --warmup 1 > gpurun_out/exp_$1_$2.json 2>/dev/null \
    && python -c "import json;d=json.load(open('gpurun_out/exp_$1_$2.json'));print('W=$1 SEG=$2', d['roofline']['kernel_ms'], d['ms_per_step'])" \
    || echo "W=$1 SEG=$2 failed"
done
