#!/bin/bash
# Kernel trace + stats of the config-4 bench leg only (quick A/B of the non-FFD kernels).
# Usage (on the GPU box): tools/ktrace.sh <tag> [extra bench args]  -> gpurun_out/kt_<tag>/
set -eo pipefail
tag=${1:?tag}; shift
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/kt_$tag
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- \
  python3 "$root/bench.py" --no-cpu-baseline --no-legs --no-stage2 --steps 2 --warmup 1 "$@" > "$out/log.txt" 2>&1
f=$(find "$out" -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(f"{float(r['AverageNs'])/1e6:9.3f} ms x{r['Calls']:>3}  {r['Name'][:110]}")
PY
