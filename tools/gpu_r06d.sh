#!/bin/bash
# class engine: parity tests, stamps, bench lines (c3 c2 c4)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06d}
timeout -k 10 600 python -u -m pytest tests/test_class_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1; rc=$?
tail -5 gpurun_out/${T}_tests.txt
[ $rc -eq 0 ] || { grep -E "FAILED|Error|error" gpurun_out/${T}_tests.txt | head -20; exit $rc; }
for W in c2 c3 c4; do
  timeout -k 10 300 python -u tools/cls_stamps.py $W >> gpurun_out/${T}_cls_stamps.txt 2>&1 || { tail -20 gpurun_out/${T}_cls_stamps.txt; exit 1; }
done
cat gpurun_out/${T}_cls_stamps.txt
for W in c3 c2 c4; do
FIT_ENGINE=class timeout -k 10 300 python -u bench.py --workload $W --no-cpu --no-live-pmc --no-shard-price --no-device-path --steps 5 --repeats 1 > gpurun_out/${T}_$W.json 2> gpurun_out/${T}_$W.err || { tail -5 gpurun_out/${T}_$W.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$W.json')); print('$W', d['value'], d['ms_per_step'], json.dumps(d['kernels']))"
done
