#!/bin/bash
# Session check: GPU tests, smoke, C3 bench, then the stamps breakdown of the C3 commit.
set -o pipefail
TAG=${1:-r02s}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { cat gpurun_out/${TAG}_smoke.txt; exit 1; }
timeout -k 10 300 python -u bench.py > gpurun_out/${TAG}_c3_bench.json 2> gpurun_out/${TAG}_c3_bench.err || { tail -20 gpurun_out/${TAG}_c3_bench.err; exit 1; }
cat gpurun_out/${TAG}_c3_bench.json
timeout -k 10 200 python -u tools/mw_stamps.py c3 > gpurun_out/${TAG}_stamps.txt 2>&1 || exit 1
head -8 gpurun_out/${TAG}_stamps.txt
echo ok
