#!/bin/bash
# write-through scan outputs: parity (full suite) + stamps + A/B vs the double-buffered build
set -o pipefail
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_full.sh ${TAG} || exit 1
timeout -k 10 200 python -u tools/mw_stamps.py c3 libfitgpu_stampsns.so > gpurun_out/${TAG}_c3_stamps.txt 2>&1 || { tail -20 gpurun_out/${TAG}_c3_stamps.txt; exit 1; }
grep -v "comp " gpurun_out/${TAG}_c3_stamps.txt
FITGPU_STAMPS_LIB=$PWD/slurm-bridge-operator_amd/fitgpu/libfitgpu_stampsns.so timeout -k 10 200 python -u tools/tl_stamps.py > gpurun_out/${TAG}_c5_tlstamps.txt 2>&1 || { tail -20 gpurun_out/${TAG}_c5_tlstamps.txt; exit 1; }
grep -v "comp " gpurun_out/${TAG}_c5_tlstamps.txt
bash tools/gpu_abx.sh ${TAG} "c3 c2 c5" 2 wt main
