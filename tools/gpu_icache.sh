#!/bin/bash
# Instruction-cache counters of the dominant kernels (one rocprofv3 --pmc pass each).
set -o pipefail
TAG=${1:-r03i}
export TMPDIR=/tmp
mkdir -p gpurun_out
P="--no-cpu --no-live-pmc --no-shard-price --repeats 1 --no-device-path"
for w in c3 c5; do
  timeout -s KILL 150 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE --output-format csv -d gpurun_out/${TAG}_icache_$w -o pmc -- python3 bench.py --workload $w --steps 1 --warmup 1 $P > gpurun_out/${TAG}_icache_$w.out 2>&1 || { echo "$w icache pass failed"; tail -5 gpurun_out/${TAG}_icache_$w.out; exit 1; }
done
echo ok
