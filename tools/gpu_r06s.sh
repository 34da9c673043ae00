#!/bin/bash
# class-engine stamps: per-segment decider cycles (tools/cls_stamps.py) on c2 / c3 / c4
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06s}
for W in ${2:-c2 c3 c4}; do
  timeout -k 10 300 python -u tools/cls_stamps.py $W >> gpurun_out/${T}_cls_stamps.txt 2>&1 || { tail -20 gpurun_out/${T}_cls_stamps.txt; exit 1; }
done
cat gpurun_out/${T}_cls_stamps.txt
