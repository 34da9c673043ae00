#!/bin/bash
# bench one workload under several values of one env knob: sweep_env2.sh TAG WL VAR v1 v2 ...
set -o pipefail
TAG=$1; WL=$2; VAR=$3; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python -u bench.py --workload $WL --no-cpu --steps 5 --warmup 2 > gpurun_out/${TAG}_${WL}_$v.json 2> gpurun_out/${TAG}_${WL}_$v.err || { tail -20 gpurun_out/${TAG}_${WL}_$v.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_${WL}_$v.json'));k=list(d['kernels'].values())[0];print('$WL $VAR=$v', round(d['value']), d['ms_per_step'], k['ms_per_launch'], d['rounds_per_step'], d['round_stops_per_step'])"
done
