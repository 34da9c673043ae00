#!/bin/bash
# Live-job commit, helpers' tile hand-off in SGPRs: parity (C3 + C5 engines), A/B main / noskip.
set -o pipefail
TAG=${1:-r03c}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_place_gpu.py tests/test_fuzz_gpu.py tests/test_golden_gpu.py tests/test_timeline_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { tail -40 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tests.txt
bash tools/gpu_ab.sh ${TAG}ab3 c3 tests/test_golden_gpu.py main noskip || exit 1
bash tools/gpu_ab.sh ${TAG}ab2 c2 tests/test_golden_gpu.py main noskip || exit 1
bash tools/gpu_ab.sh ${TAG}ab3o c3o tests/test_golden_gpu.py main noskip || exit 1
bash tools/gpu_ab.sh ${TAG}ab5 c5 tests/test_golden_gpu.py main || exit 1
timeout -k 10 200 python -u tools/mw_stamps.py c3 > gpurun_out/${TAG}_stamps.txt 2>&1; cat gpurun_out/${TAG}_stamps.txt
echo ok
