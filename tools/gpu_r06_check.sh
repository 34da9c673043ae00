#!/bin/bash
# Round 6: the admission kernel's GPU tests and bench line, then a wide fuzz sweep over every
# engine (tools/fuzz_sweep.py) at the current HEAD.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06t}
timeout -k 10 400 python -u -m pytest tests/test_direct_gpu.py tests/test_admit_gpu.py tests/test_callsite_gpu.py tests/test_fuzz_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_tests.txt
timeout -k 10 300 python -u bench.py --workload admit > gpurun_out/${T}_admit_bench.json 2> gpurun_out/${T}_admit_bench.err || { tail -20 gpurun_out/${T}_admit_bench.err; exit 1; }
python3 -c "
import json
d = json.load(open('gpurun_out/${T}_admit_bench.json'))
print({k: (v['p50_us'], v['p99_us'], v['pods_per_s']) for k, v in d['policies'].items()})
print(d['batch_split'])
"
timeout -k 10 900 python -u tools/fuzz_sweep.py ${2:-50000} ${3:-52000} > gpurun_out/${T}_fuzz_sweep.txt 2>&1; rc=$?
tail -2 gpurun_out/${T}_fuzz_sweep.txt
exit $rc
