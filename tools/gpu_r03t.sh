#!/bin/bash
set -eo pipefail
root=${GRAFT_REPO_ROOT:-$(pwd)}
out=$root/gpurun_out/lvl_trace
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d "$out" -o run -- python3 "$root/tools/lvl_time.py" > "$out/log.txt" 2>&1
f=$(find "$out" -name '*kernel_stats.csv' | head -1)
python3 - "$f" <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(f"{float(r['AverageNs'])/1e6:9.4f} ms x{r['Calls']:>3}  {r['Name'][:100]}")
PY
