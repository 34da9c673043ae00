#!/bin/bash
# round-start stamps (C3 / C5), TM_PREP parity + paired A/B on C5, UCAP 64 A/B on C3 / C2
set -o pipefail
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
L=$PWD/slurm-bridge-operator_amd/fitgpu
timeout -k 10 200 python -u tools/mw_stamps.py c3 libfitgpu_stampsns.so > gpurun_out/${TAG}_c3_stamps.txt 2>&1 || { tail -20 gpurun_out/${TAG}_c3_stamps.txt; exit 1; }
grep -v "comp " gpurun_out/${TAG}_c3_stamps.txt
FITGPU_STAMPS_LIB=$L/libfitgpu_stampsns.so timeout -k 10 200 python -u tools/tl_stamps.py > gpurun_out/${TAG}_c5_tlstamps.txt 2>&1 || { tail -20 gpurun_out/${TAG}_c5_tlstamps.txt; exit 1; }
grep -v "comp " gpurun_out/${TAG}_c5_tlstamps.txt
FITGPU_LIB=$L/libfitgpu_prep.so timeout -k 10 400 python -u -m pytest tests/test_timeline_gpu.py tests/test_golden_big_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_prep_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_prep_tests.txt; exit 1; }
tail -1 gpurun_out/${TAG}_prep_tests.txt
bash tools/gpu_abx.sh ${TAG} "c5" 3 main prep && bash tools/gpu_abx.sh ${TAG}u "c3 c2" 2 main u64
