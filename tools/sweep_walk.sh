#!/bin/bash
# C5 walk-threshold sweep: bench each variant library built with
#   make -C slurm-bridge-operator_amd fullvariant V=ww<N> DEFS="-DTL_WAVE_WALKS=<N>"
# usage: bash tools/sweep_walk.sh ww0 ww12 ...
set -o pipefail
mkdir -p gpurun_out
for v in "$@"; do
  FITGPU_LIB=$GRAFT_REPO_ROOT/slurm-bridge-operator_amd/fitgpu/libfitgpu_$v.so timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > gpurun_out/sweep_$v.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/sweep_$v.json'));print('$v', d['value'], d['ms_per_step'])"
done
