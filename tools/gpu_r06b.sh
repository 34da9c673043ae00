#!/bin/bash
# Round 6: the class engine's parity tests (tests/test_class_gpu.py), then a C3 bench line with it.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06b}
timeout -k 10 600 python -u -m pytest tests/test_class_gpu.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1; rc=$?
tail -25 gpurun_out/${T}_tests.txt
[ $rc -eq 0 ] || exit $rc
for W in c3 c2 c4; do
FIT_ENGINE=class timeout -k 10 300 python -u bench.py --workload $W --no-cpu --no-live-pmc --no-shard-price --no-device-path --steps 5 --repeats 1 > gpurun_out/${T}_$W.json 2> gpurun_out/${T}_$W.err || { tail -5 gpurun_out/${T}_$W.err; exit 1; }
python3 -c "
import json; d=json.load(open('gpurun_out/${T}_$W.json')); print('$W', d['value'], d['ms_per_step'], json.dumps(d['kernels']))"
done
