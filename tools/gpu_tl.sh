#!/bin/bash
# C5 iteration: timeline parity tests, bench, stamps (diagnostic build)
set -o pipefail
T=${1:-tl}
timeout -k 10 400 python -u -m pytest tests/test_timeline_gpu.py -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.log 2>&1 || { tail -30 gpurun_out/${T}_tests.log; exit 1; }
tail -2 gpurun_out/${T}_tests.log
timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > gpurun_out/${T}_bench.json 2>/dev/null || exit 1
python -c "import json;d=json.load(open('gpurun_out/${T}_bench.json'));print(d['value'], d['ms_per_step'], d['rounds_per_step'], d['round_stops_per_step'], {k:v['ms_per_launch'] for k,v in d['kernels'].items()})"
timeout -k 10 200 python -u tools/tl_stamps.py > gpurun_out/${T}_stamps.txt 2>&1; cat gpurun_out/${T}_stamps.txt
if [ -n "$2" ]; then
  FITGPU_LIB=$GRAFT_REPO_ROOT/slurm-bridge-operator_amd/fitgpu/libfitgpu_$2.so timeout -k 10 300 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > gpurun_out/${T}_bench_$2.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/${T}_bench_$2.json'));print('$2', d['value'], d['ms_per_step'], d['rounds_per_step'], d['round_stops_per_step'], {k:v['ms_per_launch'] for k,v in d['kernels'].items()})"
fi
