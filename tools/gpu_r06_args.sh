#!/bin/bash
# Round 6: small batches in k_small's kernel arguments (FIT_SMALL_ARGS) and the spinning
# completion wait (FIT_SYNC_SPIN): the admission GPU tests, then the bench's batch split and the
# native-caller admission line for each switch setting.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06v}
timeout -k 10 400 python -u -m pytest tests/test_direct_gpu.py tests/test_admit_gpu.py tests/test_callsite_gpu.py tests/test_fuzz_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
for cfg in "1 1" "0 1" "1 0" "0 0" "1 1"; do
  set -- $cfg
  FIT_SMALL_ARGS=$1 FIT_SYNC_SPIN=$2 timeout -k 10 300 python -u bench.py --workload admit > gpurun_out/${T}_admit_$1$2.json 2> gpurun_out/${T}_admit_$1$2.err || { tail -5 gpurun_out/${T}_admit_$1$2.err; exit 1; }
  python3 -c "
import json, sys
d = json.load(open('gpurun_out/${T}_admit_$1$2.json'))
print('args=$1 spin=$2', {k: (v['p50_us'], v['p99_us'], v['pods_per_s']) for k, v in d['policies'].items()},
      {t: {b: r['call_us_p50'] for b, r in v.items()} for t, v in d['batch_split'].items()})
"
done
