#!/bin/bash
# Round-end check, part 2: rocprofv3 kernel-trace summaries and PMC passes (tools/gpu_profile.sh),
# then the C5 decider split by phase (fine stamps build, diagnostic).
set -o pipefail
TAG=${1:-final}
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_profile.sh ${TAG} || exit 1
FITGPU_STAMPS_LIB=$PWD/slurm-bridge-operator_amd/fitgpu/libfitgpu_tlfine.so timeout -k 10 300 python -u tools/tl_stamps.py > gpurun_out/${TAG}_c5_tlfine.txt 2>&1 || { tail -20 gpurun_out/${TAG}_c5_tlfine.txt; exit 1; }
grep -v "comp " gpurun_out/${TAG}_c5_tlfine.txt
echo ok
