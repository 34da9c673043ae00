#!/bin/bash
# One GPU call: parity tests, bench line, rocprof kernel-trace summary.  Every GPU step has its own
# time limit and the steps are chained with && so the first failure ends the call.
set -o pipefail
TAG=${1:-r01}
mkdir -p gpurun_out
cd "$GRAFT_REPO_ROOT" 2>/dev/null || true
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_pytest_gpu.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_prof -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/${TAG}_prof_bench.json 2> gpurun_out/${TAG}_prof.err
rc=$?
echo "rc=$rc"
tail -3 gpurun_out/${TAG}_pytest_gpu.log
cat gpurun_out/${TAG}_bench.json
find gpurun_out/${TAG}_prof -name '*kernel_stats.csv' -exec cat {} \;
exit $rc
