#!/bin/bash
# gpurun with retries while the pool has no free box (exit 3, or a transient
# infrastructure failure before anything ran); any other outcome ends it.
# usage: gpurun_retry.sh LOG TIMEOUT 'command'
LOG=$1; T=$2; shift 2
for i in $(seq 1 20); do
  /usr/local/graft/bin/gpurun --timeout "$T" -- "$@" > "$LOG" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$LOG"; then sleep 75; continue; fi
  exit $rc
done
exit $rc
