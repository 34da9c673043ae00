#!/bin/bash
# Full -m gpu suite (one process, per-test timeout) then smoke(); output under gpurun_out/.
set -o pipefail
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -3 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 180 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { cat gpurun_out/${TAG}_smoke.txt; exit 1; }
tail -2 gpurun_out/${TAG}_smoke.txt
echo ok
