#!/bin/bash
# Round 6: VERDICT r5 item 4 — the direct small placement fused into one kernel (k_small: prefilter
# + job order + placement) with one packed H2D and one D2H copy per batch: its GPU tests, the
# admission bench line with its batch split and the one-partition (one VK's engine) variant, and
# the rocprofv3 kernel trace of what CreatePod runs.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06k}
timeout -k 10 400 python -u -m pytest tests/test_direct_gpu.py tests/test_admit_gpu.py tests/test_callsite_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_tests.txt
timeout -k 10 300 python -u bench.py --workload admit > gpurun_out/${T}_admit_bench.json 2> gpurun_out/${T}_admit_bench.err || { tail -20 gpurun_out/${T}_admit_bench.err; exit 1; }
cat gpurun_out/${T}_admit_bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_admit_prof -o run -- python3 bench.py --workload admit --admit-pods 100 > /dev/null 2> gpurun_out/${T}_admit_prof.err || { tail -20 gpurun_out/${T}_admit_prof.err; exit 1; }
echo done
