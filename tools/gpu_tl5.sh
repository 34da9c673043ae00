#!/bin/bash
# C5 diagnostics: k_commit_tl stamps, then the C5 bench per library variant (base + args).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${T:-tl5}
timeout -k 10 200 python -u tools/tl_stamps.py > gpurun_out/${T}_stamps.txt 2>&1 || { tail -5 gpurun_out/${T}_stamps.txt; exit 1; }
cat gpurun_out/${T}_stamps.txt
for v in base "$@"; do
  L=slurm-bridge-operator_amd/fitgpu/libfitgpu_$v.so
  [ "$v" = base ] && L=slurm-bridge-operator_amd/fitgpu/libfitgpu.so
  FITGPU_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --workload c5 --no-cpu --steps 3 --warmup 1 > gpurun_out/${T}_$v.json 2> gpurun_out/${T}_$v.err || { tail -5 gpurun_out/${T}_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_$v.json'));k=list(d['kernels'].values())[0];print('$v', d['value'], k['ms_per_launch'], d['rounds_per_step'], d['round_stops_per_step'])"
done
