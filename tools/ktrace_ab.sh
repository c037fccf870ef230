#!/bin/bash
# Kernel-trace the config-4 leg for several library variants and print the named kernels.
# Usage (GPU box): tools/ktrace_ab.sh <tag> <kernel-regex> <suffix>...  (suffix default = libfleetplace.so)
set -o pipefail
tag=${1:?tag}; re=${2:?regex}; shift 2
root=${GRAFT_REPO_ROOT:-$(pwd)}
for v in "$@"; do
  lib=$root/fleetflow_amd/libfleetplace${v#default}.so
  FLEETPLACE_LIB=$lib bash "$root/tools/ktrace.sh" "${tag}_$v" > /dev/null || { echo "variant $v failed"; exit 1; }
  f=$(find "$root/gpurun_out/kt_${tag}_$v" -name '*kernel_stats.csv' | head -1)
  python3 - "$f" "$v" "$re" <<'PY'
import csv, re, sys
for r in csv.DictReader(open(sys.argv[1])):
    if re.search(sys.argv[3], r['Name']):
        print(f"{sys.argv[2]:>10} {float(r['AverageNs'])/1e6:8.3f} ms x{r['Calls']:>3} {r['Name'][:70]}")
PY
done
