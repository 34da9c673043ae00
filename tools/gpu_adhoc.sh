set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02g}
timeout -k 10 60 python -u tools/decbench.py > gpurun_out/${T}_decbench.txt 2>&1 || { cat gpurun_out/${T}_decbench.txt; exit 1; }
cat gpurun_out/${T}_decbench.txt
timeout -k 10 120 python -u tools/mw_stamps.py c3 > gpurun_out/${T}_stamps.txt 2>&1 || { tail gpurun_out/${T}_stamps.txt; exit 1; }
head -5 gpurun_out/${T}_stamps.txt
timeout -k 10 300 python -u -m pytest tests/test_place_gpu.py tests/test_golden_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_tests.txt
for v in "" idle4; do
  L=slurm-bridge-operator_amd/fitgpu/libfitgpu${v:+_$v}.so
  FITGPU_LIB=$PWD/$L timeout -k 10 120 python -u bench.py --no-cpu --no-device-path > gpurun_out/${T}_c3_${v:-base}.json 2>&1 || { tail -5 gpurun_out/${T}_c3_${v:-base}.json; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().splitlines()[-1]); print(sys.argv[1], d['value'], d['ms_per_step'], d['kernels'])" gpurun_out/${T}_c3_${v:-base}.json
done
