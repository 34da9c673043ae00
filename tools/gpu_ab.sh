#!/bin/bash
# A/B of in-tree library variants (fitgpu/libfitgpu_<v>.so, FITGPU_LIB) on one workload: parity
# tests of the workload's engine, then a short bench line per variant.  Usage:
#   tools/gpu_ab.sh TAG WORKLOAD TESTFILE variant...   ("main" = fitgpu/libfitgpu.so)
set -o pipefail
TAG=$1; WL=$2; TF=$3; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  if [ "$v" = main ]; then L=slurm-bridge-operator_amd/fitgpu/libfitgpu.so; else L=slurm-bridge-operator_amd/fitgpu/libfitgpu_$v.so; fi
  FITGPU_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest $TF -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_${v}_tests.txt 2>&1 || { echo "$v tests failed"; tail -30 gpurun_out/${TAG}_${v}_tests.txt; exit 1; }
  tail -1 gpurun_out/${TAG}_${v}_tests.txt
  FITGPU_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --workload $WL --steps 10 --warmup 2 --repeats 1 --no-cpu --no-live-pmc --no-shard-price --no-device-path > gpurun_out/${TAG}_${v}_bench.json 2> gpurun_out/${TAG}_${v}_bench.err || { echo "$v bench failed"; tail -20 gpurun_out/${TAG}_${v}_bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_${v}_bench.json')); k=list(d['kernels'].values())[0]; print('$v', d['value'], d['ms_per_step'], k['ms_per_launch'], d['rounds_per_step'], d['round_stops_per_step'])"
done
echo ok
