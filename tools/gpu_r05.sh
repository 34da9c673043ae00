#!/bin/bash
# Round 5 check: the full -m gpu suite and smoke, the admission A/B (small batches on the
# host-driven rounds vs the persistent engine), the C4 line with its rocprof kernel summary, and a
# quick C3 line.  Every GPU step has its own limit; the first failure ends the call.
set -o pipefail
TAG=${1:-r05b}
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_full.sh ${TAG} || exit 1
Q="--no-cpu --no-live-pmc --no-shard-price"
FIT_SMALL_BATCH=-1 timeout -k 10 300 python -u bench.py --workload admit > gpurun_out/${TAG}_admit_persistent.json 2> gpurun_out/${TAG}_admit_persistent.err || { tail -20 gpurun_out/${TAG}_admit_persistent.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload admit > gpurun_out/${TAG}_admit_bench.json 2> gpurun_out/${TAG}_admit_bench.err || { tail -20 gpurun_out/${TAG}_admit_bench.err; exit 1; }
timeout -k 10 600 python -u bench.py --workload c4 > gpurun_out/${TAG}_c4_bench.json 2> gpurun_out/${TAG}_c4_bench.err || { tail -20 gpurun_out/${TAG}_c4_bench.err; exit 1; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c4_prof -o run -- python3 bench.py --workload c4 --steps 5 --warmup 2 $Q --repeats 1 --no-device-path > /dev/null 2>gpurun_out/${TAG}_c4_prof.err || exit 1
timeout -k 10 300 python -u bench.py $Q > gpurun_out/${TAG}_c3_quick.json 2> gpurun_out/${TAG}_c3_quick.err || { tail -20 gpurun_out/${TAG}_c3_quick.err; exit 1; }
for f in admit_persistent admit_bench c4_bench c3_quick; do echo "== $f"; cut -c1-600 gpurun_out/${TAG}_$f.json; done
echo ok
