set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02j}
timeout -k 10 60 python -u tools/decbench.py > gpurun_out/${T}_decbench.txt 2>&1 || { cat gpurun_out/${T}_decbench.txt; exit 1; }
tail -1 gpurun_out/${T}_decbench.txt
timeout -k 10 400 python -u -m pytest tests/test_place_gpu.py tests/test_golden_gpu.py tests/test_e2e_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
for v in stamps st_xor st_noprio; do
  timeout -k 10 120 python -u tools/mw_stamps.py c3 libfitgpu_$v.so > gpurun_out/${T}_$v.txt 2>&1 || { tail gpurun_out/${T}_$v.txt; exit 1; }
  echo "== $v"; head -2 gpurun_out/${T}_$v.txt
done
