#!/bin/bash
# C3 iteration: placement parity tests, bench, decider/helper stamps (diagnostic build)
set -o pipefail
T=${1:-c3}
timeout -k 10 500 python -u -m pytest tests/test_place_gpu.py tests/test_golden_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u bench.py --workload c3 --steps 5 --warmup 2 --no-cpu > gpurun_out/${T}_bench.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/${T}_bench.json'));print(d['value'], d['ms_per_step'], d['rounds_per_step'], d['round_stops_per_step'], {k:v['ms_per_launch'] for k,v in d['kernels'].items()})"
timeout -k 10 200 python -u tools/mw_stamps.py > gpurun_out/${T}_stamps.txt 2>&1; head -3 gpurun_out/${T}_stamps.txt
