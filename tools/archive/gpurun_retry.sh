#!/bin/bash
# Retry a gpurun call while the pool has no free box (exit 3: nothing ran, nothing charged) or the box
# was lost before the command started (status=transient, rc=None). Any other outcome is final.
#   bash tools/gpurun_retry.sh <outfile> <timeout> <command...>
OUT=$1; shift
TO=$1; shift
for i in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$@" > "$OUT" 2>&1
  RC=$?
  if [ $RC -eq 3 ] || grep -q "status=transient rc=None" "$OUT"; then
    echo "attempt $i: no box ($RC), retrying in 150 s" >> "$OUT.retries"
    sleep 150
    continue
  fi
  exit $RC
done
exit 3
