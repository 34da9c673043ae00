#!/bin/bash
# Bench-only A/B of in-tree library variants, interleaved (v1 v2 v1 v2 ...) per workload, so box
# drift shows up.  Usage: tools/gpu_abx.sh TAG "WORKLOADS" ROUNDS variant...  ("main" = libfitgpu.so)
set -o pipefail
TAG=$1; WLS=$2; NR=$3; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in $WLS; do
  for r in $(seq 1 $NR); do
    for v in "$@"; do
      if [ "$v" = main ]; then L=slurm-bridge-operator_amd/fitgpu/libfitgpu.so; else L=slurm-bridge-operator_amd/fitgpu/libfitgpu_$v.so; fi
      FITGPU_LIB=$PWD/$L timeout -k 10 300 python -u bench.py --workload $wl --steps 10 --warmup 2 --repeats 1 --no-cpu --no-live-pmc --no-shard-price --no-device-path > gpurun_out/${TAG}_${wl}_${v}_$r.json 2> gpurun_out/${TAG}_${wl}_${v}_$r.err || { echo "$v bench failed"; tail -20 gpurun_out/${TAG}_${wl}_${v}_$r.err; exit 1; }
      python -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_${wl}_${v}_$r.json')); k=list(d['kernels'].values())[0]; print('$wl $v', d['value'], d['ms_per_step'], k['ms_per_launch'], d['rounds_per_step'], d['round_stops_per_step'])"
    done
  done
done
echo ok
