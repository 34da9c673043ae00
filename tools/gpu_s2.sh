#!/bin/bash
# Session check: GPU tests, smoke, bench lines (C3, C5), the C3 stamps breakdown, decider alone.
set -o pipefail
TAG=${1:-r02t}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/${TAG}_gpu_tests.txt 2>&1 || { tail -30 gpurun_out/${TAG}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${TAG}_gpu_tests.txt
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.txt 2>&1 || { cat gpurun_out/${TAG}_smoke.txt; exit 1; }
for w in c3 c5; do
  timeout -k 10 300 python -u bench.py --workload $w > gpurun_out/${TAG}_${w}_bench.json 2> gpurun_out/${TAG}_${w}_bench.err || { tail -20 gpurun_out/${TAG}_${w}_bench.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/${TAG}_${w}_bench.json'));print('$w', d['value'], d['ms_per_step'], d['kernel_path_value'], list(d['kernels'].values())[0]['ms_per_launch'])"
done
timeout -k 10 200 python -u tools/mw_stamps.py c3 > gpurun_out/${TAG}_stamps.txt 2>&1 || exit 1
head -6 gpurun_out/${TAG}_stamps.txt
timeout -k 10 100 python -u tools/decbench.py > gpurun_out/${TAG}_decbench.txt 2>&1 || exit 1
cat gpurun_out/${TAG}_decbench.txt
echo ok
