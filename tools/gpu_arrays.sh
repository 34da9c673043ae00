#!/bin/bash
# Array-expanded queues: parity tests, then one bench line per array workload (and the plain
# workload beside it for comparison).  Usage: tools/gpu_arrays.sh TAG
set -o pipefail
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_arrays_gpu.py -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -3 gpurun_out/${TAG}_tests.txt
for wl in c2a c2 c3a c5a; do
  timeout -k 10 400 python -u bench.py --workload $wl --steps 10 --warmup 2 --repeats 3 --no-live-pmc --no-shard-price --no-cpu > gpurun_out/${TAG}_${wl}_bench.json 2> gpurun_out/${TAG}_${wl}_bench.err || { echo "$wl bench failed"; tail -20 gpurun_out/${TAG}_${wl}_bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_${wl}_bench.json')); k=list(d['kernels'].values())[0]; print('$wl', d['value'], d['ms_per_step'], k['ms_per_launch'], d['rounds_per_step'], d['round_stops_per_step'], d['jobs'])"
done
echo ok
