#!/bin/bash
# Round-3 check: timeline parity first (the new decider/helper commit), then every -m gpu test,
# smoke, bench lines and the C5 stamps breakdown.  Each GPU step has its own limit; the first
# failure ends the call.
set -o pipefail
TAG=${1:-r03}
shift
WL=${@:-c5 c3}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_timeline_gpu.py tests/test_admit_gpu.py tests/test_concurrent_gpu.py -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tl_tests.txt 2>&1 || { tail -40 gpurun_out/${TAG}_tl_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tl_tests.txt
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { cat gpurun_out/${TAG}_smoke.txt; exit 1; }
for w in $WL; do
  timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/${TAG}_${w}_bench.json 2> gpurun_out/${TAG}_${w}_bench.err || { tail -20 gpurun_out/${TAG}_${w}_bench.err; exit 1; }
  cut -c1-600 gpurun_out/${TAG}_${w}_bench.json
done
timeout -k 10 200 python -u tools/tl_stamps.py > gpurun_out/${TAG}_tlstamps.txt 2>&1; cat gpurun_out/${TAG}_tlstamps.txt
echo ok
