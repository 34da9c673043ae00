#!/bin/bash
# C3 commit-knob sweep: stamps breakdown, then the bench per prebuilt variant library
# (make -C slurm-bridge-operator_amd variant V=<name> DEFS="-D...").  Every GPU step is time-limited.
set -o pipefail
T=${T:-sw}
WL=${WL:-c3}
timeout -k 10 200 python -u tools/mw_stamps.py $WL > gpurun_out/${T}_stamps.txt 2>&1 || exit 1
head -6 gpurun_out/${T}_stamps.txt
for v in base "$@"; do
  lib=slurm-bridge-operator_amd/fitgpu/libfitgpu_$v.so
  [ "$v" = base ] && lib=slurm-bridge-operator_amd/fitgpu/libfitgpu.so
  FITGPU_LIB=$PWD/$lib timeout -k 10 200 python -u bench.py --workload $WL --steps 5 --warmup 2 --no-cpu > gpurun_out/${T}_$v.json 2>gpurun_out/${T}_$v.err || { tail -5 gpurun_out/${T}_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_$v.json'));print('$v', d['value'], d['ms_per_step'], d['rounds_per_step'], list(d['kernels'].values())[0]['ms_per_launch'], d['round_stops_per_step'])"
done
