#!/bin/bash
# gpurun with retries only when no box was obtained (exit 3: nothing ran, nothing charged)
LOG=$1; shift
for k in 1 2 3 4 5 6; do
  /usr/local/graft/bin/gpurun "$@" > $LOG 2>&1; rc=$?
  [ $rc -ne 3 ] && exit $rc
  sleep 90
done
exit 3
