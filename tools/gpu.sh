#!/bin/bash
# Run a command on the GPU box via gpurun; retry ONLY when gpurun reports that the
# box never ran it (status=transient / exit 3), at most 8 attempts, sleeping for the
# back-off gpurun advertises ("retry in Ns").  A command that ran and failed is never
# retried.
set -u
for attempt in 1 2 3 4 5 6 7 8; do
  out=$(/usr/local/graft/bin/gpurun "$@" 2>&1); rc=$?
  echo "$out" | tail -4
  if echo "$out" | grep -q "status=transient" || [ $rc -eq 3 ]; then
    wait_s=$(echo "$out" | grep -o 'retry in [0-9]*s' | grep -o '[0-9]*' | tail -1)
    wait_s=${wait_s:-60}
    echo "[gpu.sh] infrastructure not ready (attempt $attempt), waiting $((wait_s + 10)) s"
    sleep $((wait_s + 10)); continue
  fi
  exit $rc
done
exit 3
