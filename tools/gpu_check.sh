#!/bin/bash
# GPU check of the tree: -m gpu tests (one process, per-test timeout), smoke(), then bench lines.
# Every GPU step has its own limit; the first failure ends the call.
set -o pipefail
TAG=${1:-r02}
shift
WL=${@:-c3}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -3 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { cat gpurun_out/${TAG}_smoke.txt; exit 1; }
for w in $WL; do
  timeout -k 10 300 python -u bench.py --workload $w > gpurun_out/${TAG}_${w}_bench.json 2> gpurun_out/${TAG}_${w}_bench.err || { tail -20 gpurun_out/${TAG}_${w}_bench.err; exit 1; }
  cat gpurun_out/${TAG}_${w}_bench.json
done
echo ok
