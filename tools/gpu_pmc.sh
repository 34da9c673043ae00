#!/bin/bash
# PMC passes for the dominant kernel (one rocprofv3 run per counter group; MI355X_MICROARCH.md
# "rocprofv3 PMC slots": FETCH_SIZE and WRITE_SIZE cannot share a pass).
set -o pipefail
TAG=${1:-r01}
ARGS=${2:-"--steps 2 --warmup 1 --no-cpu"}
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/${TAG}_pmc$i -o pmc -- python3 bench.py $ARGS > gpurun_out/${TAG}_pmc$i.out 2>&1 || { echo "pass $i ($ctr) failed"; tail -5 gpurun_out/${TAG}_pmc$i.out; exit 1; }
done
echo ok
