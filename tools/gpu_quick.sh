#!/bin/bash
# Quick GPU check after a kernel change: parity tests of the placement paths, then bench lines
# (no CPU baseline) for the given workloads.  Every GPU step has its own limit.
set -o pipefail
TAG=${1:-q}
shift
WL=${@:-c3}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_place_gpu.py tests/test_timeline_gpu.py tests/test_golden_gpu.py -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_tests.txt
for w in $WL; do
  timeout -k 10 300 python -u bench.py --workload $w --no-cpu > gpurun_out/${TAG}_${w}.json 2> gpurun_out/${TAG}_${w}.err || { tail -20 gpurun_out/${TAG}_${w}.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_${w}.json'));k=list(d['kernels'].values())[0];print('$w', d['value'], d['ms_per_step'], d['kernel_path_value'], k['ms_per_launch'], d['rounds_per_step'], d['round_stops_per_step'])"
done
