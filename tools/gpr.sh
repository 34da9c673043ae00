#!/bin/bash
# gpurun, retried only when the call never ran on a box (no box / slot free, or the box was lost
# before the command started: gpurun reports status=transient and charges nothing)
LOG=$1; shift
for k in $(seq 1 ${GPR_TRIES:-8}); do
  /usr/local/graft/bin/gpurun "$@" > $LOG 2>&1; rc=$?
  grep -q "status=transient" $LOG || exit $rc
  sleep 60
done
exit 3
