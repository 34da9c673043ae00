#!/bin/bash
# C3 bench under engine environment knobs: each argument is one "VAR=value ..." setting
set -o pipefail
T=${T:-se}
i=0
for env in "" "$@"; do
  i=$((i+1))
  env $env timeout -k 10 200 python -u bench.py --workload ${WL:-c3} --steps ${STEPS:-5} --warmup 2 --no-cpu > gpurun_out/${T}_$i.json 2>gpurun_out/${T}_$i.err || { tail -5 gpurun_out/${T}_$i.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${T}_$i.json'));print('[$env]', d['value'], d['ms_per_step'], d.get('rounds_per_step'), d.get('round_stops_per_step'), list(d['kernels'].values())[0]['ms_per_launch'])"
done
