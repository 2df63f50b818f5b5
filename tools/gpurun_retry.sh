#!/bin/bash
# gpurun with retries while the pool has no free box (status=transient / exit 3:
# nothing ran, nothing charged). Any other outcome -- success or a failure of
# the command itself -- ends it: a failing GPU step is never run again.
# usage: tools/gpurun_retry.sh <log> <gpurun args...>
log=$1; shift
for i in 1 2 3 4 5 6 7 8; do
  /usr/local/graft/bin/gpurun "$@" > "$log" 2>&1
  rc=$?
  if [ $rc -eq 3 ] || grep -q "status=transient" "$log"; then sleep 150; continue; fi
  exit $rc
done
exit 3
