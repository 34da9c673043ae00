#!/bin/bash
# GPU run of selected test files (one pytest process, per-test timeout); output under gpurun_out/.
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1
rc=$?
tail -30 gpurun_out/${TAG}_tests.txt
exit $rc
