#!/bin/bash
# helper extraction early exit: parity of the default build (MW_EE=1) and of the TL variants,
# then interleaved bench lines
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_arrays_gpu.py tests/test_place_gpu.py tests/test_live_jobs_gpu.py tests/test_golden_gpu.py tests/test_fuzz_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04ee_tests.txt 2>&1 || { tail -40 gpurun_out/r04ee_tests.txt; exit 1; }
tail -1 gpurun_out/r04ee_tests.txt
for v in tee teex; do
  FITGPU_LIB=$PWD/slurm-bridge-operator_amd/fitgpu/libfitgpu_$v.so timeout -k 10 600 python -u -m pytest tests/test_timeline_gpu.py tests/test_golden_big_gpu.py -k "c5 or timeline or tl" -x -q --timeout 300 --timeout-method thread > gpurun_out/r04ee_${v}_tests.txt 2>&1 || { tail -30 gpurun_out/r04ee_${v}_tests.txt; exit 1; }
  tail -1 gpurun_out/r04ee_${v}_tests.txt
done
bash tools/gpu_abx.sh r04ee2 "c2 c3" 2 main eex && bash tools/gpu_abx.sh r04ee3 "c5" 2 main tee teex
