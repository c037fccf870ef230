#!/bin/bash
# Run a command on the GPU box via gpurun; retry ONLY when gpurun reports that the
# box never ran it (status=transient / exit 3), at most 4 attempts.  A command that
# ran and failed is never retried.
set -u
for attempt in 1 2 3 4; do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1); rc=$?
  echo "$out" | tail -4
  if echo "$out" | grep -q "status=transient" || [ $rc -eq 3 ]; then
    echo "[gpu.sh] infrastructure not ready (attempt $attempt), waiting" ; sleep 45; continue
  fi
  exit $rc
done
exit 3
