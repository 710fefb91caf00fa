#!/bin/bash
# Run one gpurun command, retrying only while the pool has no free box (exit 3: nothing ran, nothing charged).
# Any other outcome (success, a failure of the command, a refusal) is returned as is.  Usage:
#   bash scripts/gpurun_wait.sh <timeout-seconds> '<command>'
lim=$1; shift
for attempt in 1 2 3 4 5 6 7 8 9 10 11 12; do
  /usr/local/graft/bin/gpurun --timeout "$lim" -- "$@"
  rc=$?
  [ $rc -ne 3 ] && exit $rc
  echo "[gpurun_wait] no box (attempt $attempt); waiting 90 s"
  sleep 90
done
exit 3
