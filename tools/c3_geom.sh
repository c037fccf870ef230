#!/bin/bash
# Config-3 leg of bench.py under forced pipeline geometries (FLEETPLACE_PIPE_SEG groups per
# segment, FLEETPLACE_PIPE_W stages): tools/c3_geom.sh "seg:w" ...   (GPU box)
cd "${GRAFT_REPO_ROOT:-$(pwd)}" || exit 1
for g in "$@"; do
  seg=${g%%:*}; w=${g##*:}
  FLEETPLACE_PIPE_SEG=$seg FLEETPLACE_PIPE_W=$w timeout -k 10 200 python -u bench.py --no-cpu-baseline --no-stage2 \
    --steps 1 --warmup 1 --scenarios 256 --config3-steps 3 > gpurun_out/c3g_$seg_$w.json 2> gpurun_out/c3g_$seg_$w.err \
    || { echo "geom $g failed"; tail -5 gpurun_out/c3g_$seg_$w.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'c3 step', round(d['config3']['ms_per_step'],2), 'ffd', round(d['config3']['breakdown_ms']['ffd_kernel'],2))" gpurun_out/c3g_$seg_$w.json "$g"
done
