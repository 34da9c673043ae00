#!/bin/bash
# A/B of an environment knob on one workload: parity tests and a short bench line per setting.
#   tools/gpu_envab.sh TAG WORKLOAD TESTFILE "ENV=V ..." "ENV=V ..." ...   ("-" = no extra env)
set -o pipefail
TAG=$1; WL=$2; TF=$3; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out
i=0
for e in "$@"; do
  i=$((i+1)); [ "$e" = "-" ] && e=""
  env $e timeout -k 10 300 python -u -m pytest $TF -x -q --timeout 120 --timeout-method thread > gpurun_out/${TAG}_${i}_tests.txt 2>&1 || { echo "[$e] tests failed"; tail -30 gpurun_out/${TAG}_${i}_tests.txt; exit 1; }
  tail -1 gpurun_out/${TAG}_${i}_tests.txt
  env $e timeout -k 10 300 python -u bench.py --workload $WL --steps 10 --warmup 2 --repeats 1 --no-cpu --no-live-pmc --no-shard-price --no-device-path > gpurun_out/${TAG}_${i}_bench.json 2> gpurun_out/${TAG}_${i}_bench.err || { echo "[$e] bench failed"; tail -20 gpurun_out/${TAG}_${i}_bench.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/${TAG}_${i}_bench.json')); k=list(d['kernels'].values())[0]; print('[$e]', d['value'], d['ms_per_step'], k['ms_per_launch'], d['rounds_per_step'], d['round_stops_per_step'], k.get('scan_worker_busy_ms'))"
done
echo ok
