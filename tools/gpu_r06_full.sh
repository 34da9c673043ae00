#!/bin/bash
# Round 6: the whole GPU suite, smoke, then the admission bench line (box-to-box check).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06o}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -3 gpurun_out/${T}_gpu_tests.txt
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${T}_smoke.txt 2>&1 || { tail -20 gpurun_out/${T}_smoke.txt; exit 1; }
tail -3 gpurun_out/${T}_smoke.txt
timeout -k 10 300 python -u bench.py --workload admit > gpurun_out/${T}_admit_bench.json 2> gpurun_out/${T}_admit_bench.err || { tail -20 gpurun_out/${T}_admit_bench.err; exit 1; }
cat gpurun_out/${T}_admit_bench.json
