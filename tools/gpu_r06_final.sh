#!/bin/bash
# Round 6 end: every -m gpu test and smoke(), the default bench lines (C3 with CPU baselines and live
# PMC, C4 with its default engine, C5), the admission line, and rocprofv3 kernel traces of C3 / C4.
set -o pipefail
T=${1:-r06z}
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_full.sh ${T} || exit 1
for w in c3 c4 c5; do
  timeout -k 10 600 python -u bench.py --workload $w > gpurun_out/${T}_${w}_bench.json 2> gpurun_out/${T}_${w}_bench.err || { tail -20 gpurun_out/${T}_${w}_bench.err; exit 1; }
done
timeout -k 10 300 python -u bench.py --workload admit > gpurun_out/${T}_admit_bench.json 2> gpurun_out/${T}_admit_bench.err || { tail -20 gpurun_out/${T}_admit_bench.err; exit 1; }
P="--no-cpu --no-live-pmc --no-shard-price --repeats 1 --no-device-path"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c3_prof -o run -- python3 bench.py --steps 5 --warmup 2 $P > /dev/null 2>gpurun_out/${T}_c3_prof.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/${T}_c4_prof -o run -- python3 bench.py --workload c4 --steps 3 --warmup 1 $P > /dev/null 2>gpurun_out/${T}_c4_prof.err || exit 1
python3 - "$T" <<'PY'
import json, sys
t = sys.argv[1]
for w in ("c3", "c4", "c5"):
    d = json.load(open(f"gpurun_out/{t}_{w}_bench.json")); r = d["roofline"]
    print(w, d["value"], d["ms_per_step"], r["kernel"], d["kernels"][r["kernel"]]["ms_per_launch"], r["frac"], r["traffic"], (d.get("cpu_baseline") or {}).get("value"))
d = json.load(open(f"gpurun_out/{t}_admit_bench.json"))
print("admit", {k: (v["p50_us"], v["p99_us"], v["pods_per_s"]) for k, v in d["policies"].items()})
PY
echo ok
