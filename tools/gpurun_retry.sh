#!/bin/bash
# Submit one gpurun call, resubmitting ONLY when no box/slot was free (gpurun exit 3 or a "transient"
# status: nothing ran, nothing was charged).  A call that ran is never repeated.
# Usage: tools/gpurun_retry.sh <log> <timeout_s> '<command>'
LOG=$1; TO=$2; CMD=$3
for k in $(seq 1 12); do
  /usr/local/graft/bin/gpurun --timeout "$TO" -- "$CMD" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then
    echo "[retry $k] no box: waiting" >> "$LOG.retries"
    sleep 150
    continue
  fi
  exit $rc
done
exit 3
