#!/bin/bash
# Round profile: rocprofv3 kernel-trace summaries and PMC passes for the dominant kernels (C3
# k_engine, C5 k_engine_tl), plus the C2 / C3o bench lines and the admission-latency line.  The
# profiled runs use --no-live-pmc (no nested rocprofv3).  Every GPU step has its own limit; the
# first failure ends the call.
set -o pipefail
TAG=${1:-r03}
export TMPDIR=/tmp
mkdir -p gpurun_out
P="--no-cpu --no-live-pmc --no-shard-price --repeats 1 --no-device-path"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c3_prof -o run -- python3 bench.py --steps 5 --warmup 2 $P > /dev/null 2>gpurun_out/${TAG}_c3_prof.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c5_prof -o run -- python3 bench.py --workload c5 --steps 3 --warmup 1 $P > /dev/null 2>gpurun_out/${TAG}_c5_prof.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${TAG}_c4_prof -o run -- python3 bench.py --workload c4 --steps 3 --warmup 1 $P > /dev/null 2>gpurun_out/${TAG}_c4_prof.err || exit 1
i=0
for ctr in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SMEM SQ_INSTS_VMEM" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/${TAG}_pmc$i -o pmc -- python3 bench.py --steps 2 --warmup 1 $P > gpurun_out/${TAG}_pmc$i.out 2>&1 || { echo "c3 pmc pass $i failed"; exit 1; }
  timeout -s KILL 150 rocprofv3 --pmc $ctr --output-format csv -d gpurun_out/${TAG}_pmc_c5_$i -o pmc -- python3 bench.py --workload c5 --steps 1 --warmup 1 $P > gpurun_out/${TAG}_pmc_c5_$i.out 2>&1 || { echo "c5 pmc pass $i failed"; exit 1; }
done
for w in c2 c3o c4; do
  timeout -k 10 400 python -u bench.py --workload $w > gpurun_out/${TAG}_${w}_bench.json 2> gpurun_out/${TAG}_${w}_bench.err || { tail -20 gpurun_out/${TAG}_${w}_bench.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --workload admit > gpurun_out/${TAG}_admit_bench.json 2> gpurun_out/${TAG}_admit_bench.err || { tail -20 gpurun_out/${TAG}_admit_bench.err; exit 1; }
cat gpurun_out/${TAG}_admit_bench.json
echo ok
