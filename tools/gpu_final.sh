#!/bin/bash
# Round-end check, part 1: every -m gpu test and smoke(), then the default bench line (C3: CPU
# baselines, live PMC passes, node-sharding price) and the C5 line.  Part 2: tools/gpu_profile.sh.
set -o pipefail
TAG=${1:-final}
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_full.sh ${TAG} || exit 1
timeout -k 10 600 python -u bench.py > gpurun_out/${TAG}_c3_bench.json 2> gpurun_out/${TAG}_c3_bench.err || { tail -20 gpurun_out/${TAG}_c3_bench.err; exit 1; }
cat gpurun_out/${TAG}_c3_bench.json
timeout -k 10 600 python -u bench.py --workload c5 > gpurun_out/${TAG}_c5_bench.json 2> gpurun_out/${TAG}_c5_bench.err || { tail -20 gpurun_out/${TAG}_c5_bench.err; exit 1; }
cat gpurun_out/${TAG}_c5_bench.json
echo ok
