#!/bin/bash
# Round 6: the automatic class engine for multi-node queues — the GPU suite and smoke, then the C4
# bench line with its default engine choice and with FIT_CLASS=0 (the persistent engine).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06y}
bash tools/gpu_full.sh ${T} || exit 1
timeout -k 10 600 python -u bench.py --workload c4 > gpurun_out/${T}_c4_bench.json 2> gpurun_out/${T}_c4_bench.err || { tail -20 gpurun_out/${T}_c4_bench.err; exit 1; }
FIT_CLASS=0 timeout -k 10 600 python -u bench.py --workload c4 --no-cpu > gpurun_out/${T}_c4_persistent.json 2> gpurun_out/${T}_c4_persistent.err || { tail -20 gpurun_out/${T}_c4_persistent.err; exit 1; }
python3 - "$T" <<'PY'
import json, sys
t = sys.argv[1]
for f in ("c4_bench", "c4_persistent"):
    d = json.load(open(f"gpurun_out/{t}_{f}.json"))
    r = d["roofline"]
    print(f, d["value"], d["ms_per_step"], r["kernel"], d["kernels"][r["kernel"]]["ms_per_launch"], r["frac"], (d.get("cpu_baseline") or {}).get("value"))
PY
