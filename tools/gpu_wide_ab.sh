set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
FITGPU_LIB=$PWD/slurm-bridge-operator_amd/fitgpu/libfitgpu_wide.so timeout -k 10 600 python -u -m pytest tests/test_arrays_gpu.py tests/test_place_gpu.py tests/test_live_jobs_gpu.py tests/test_golden_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r04wd_tests.txt 2>&1 || { tail -30 gpurun_out/r04wd_tests.txt; exit 1; }
tail -2 gpurun_out/r04wd_tests.txt
bash tools/gpu_abx.sh r04wd "c3a c3 c2a c2 c3o" 2 main wide
