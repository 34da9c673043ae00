#!/bin/bash
# Variant sweep: for each prebuilt library (make -C slurm-bridge-operator_amd variant V=<name>
# DEFS="-D..."), the golden-digest parity tests (C1/C2/C3 full) and place tests, then the bench.
# Every GPU step is time-limited; the first failure ends the call.
set -o pipefail
T=${T:-sv}
WL=${WL:-c3}
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  lib=slurm-bridge-operator_amd/fitgpu/libfitgpu_$v.so
  [ "$v" = base ] && lib=slurm-bridge-operator_amd/fitgpu/libfitgpu.so
  FITGPU_LIB=$PWD/$lib timeout -k 10 240 python -u -m pytest ${TESTS:-tests/test_golden_gpu.py tests/test_place_gpu.py tests/test_fuzz_gpu.py} -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_${v}_tests.txt 2>&1 || { echo "$v: tests FAILED"; tail -15 gpurun_out/${T}_${v}_tests.txt; exit 1; }
  echo "$v: $(tail -1 gpurun_out/${T}_${v}_tests.txt)"
  for w in $WL; do
    FITGPU_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --workload $w --steps 5 --warmup 2 --no-cpu > gpurun_out/${T}_${v}_$w.json 2>gpurun_out/${T}_${v}_$w.err || { tail -5 gpurun_out/${T}_${v}_$w.err; exit 1; }
    python -c "import json;d=json.load(open('gpurun_out/${T}_${v}_$w.json'));print('$v $w', d['value'], d['ms_per_step'], d['rounds_per_step'], list(d['kernels'].values())[0]['ms_per_launch'], d['round_stops_per_step'])"
  done
done
