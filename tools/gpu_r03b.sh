#!/bin/bash
# Round-3 check of the live-job commit: C3-engine parity first, then an A/B of the skip
# (main vs noskip) on c3 / c2, then every -m gpu test, smoke, bench lines and stamps.
set -o pipefail
TAG=${1:-r03b}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_place_gpu.py tests/test_fuzz_gpu.py tests/test_golden_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${TAG}_c3_tests.txt 2>&1 || { tail -40 gpurun_out/${TAG}_c3_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_c3_tests.txt
bash tools/gpu_ab.sh ${TAG}ab3 c3 tests/test_golden_gpu.py main noskip || exit 1
bash tools/gpu_ab.sh ${TAG}ab2 c2 tests/test_golden_gpu.py main noskip || exit 1
bash tools/gpu_ab.sh ${TAG}ab3o c3o tests/test_golden_gpu.py main noskip || exit 1
bash tools/gpu_r03.sh ${TAG} c3 c5
