#!/bin/bash
# C5: stamps (coarse + fine, first-tile pickup) and an A/B of the tile-queue knobs.
set -o pipefail
TAG=${1:-r03d}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/tl_stamps.py > gpurun_out/${TAG}_tlstamps.txt 2>&1; cat gpurun_out/${TAG}_tlstamps.txt | grep -v "comp "
FITGPU_STAMPS_LIB=$PWD/slurm-bridge-operator_amd/fitgpu/libfitgpu_tlfine.so timeout -k 10 200 python -u tools/tl_stamps.py > gpurun_out/${TAG}_tlfine.txt 2>&1; cat gpurun_out/${TAG}_tlfine.txt | grep -v "comp "
bash tools/gpu_ab.sh ${TAG}ab5 c5 tests/test_timeline_gpu.py main prio ahead2 ahead8 || exit 1
echo ok
