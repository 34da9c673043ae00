#!/bin/bash
# Paired A/B on one box: the current build against a variant library (FITGPU_LIB), alternating,
# for the given workloads.  Usage: tools/gpu_ab_r5.sh TAG VARIANT_SO "c3 c2" [rounds]
set -o pipefail
TAG=$1; VAR=$2; WLS=${3:-c3}; N=${4:-2}
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--no-cpu --no-live-pmc --no-shard-price --no-device-path"
for i in $(seq 1 $N); do
  for w in $WLS; do
    timeout -k 10 300 python -u bench.py --workload $w $Q > gpurun_out/${TAG}_${w}_main_$i.json 2> gpurun_out/${TAG}_${w}_main_$i.err || { tail -5 gpurun_out/${TAG}_${w}_main_$i.err; exit 1; }
    FITGPU_LIB=$VAR timeout -k 10 300 python -u bench.py --workload $w $Q > gpurun_out/${TAG}_${w}_var_$i.json 2> gpurun_out/${TAG}_${w}_var_$i.err || { tail -5 gpurun_out/${TAG}_${w}_var_$i.err; exit 1; }
  done
done
python3 - "$TAG" "$WLS" "$N" <<'PY'
import json, sys
tag, wls, n = sys.argv[1], sys.argv[2].split(), int(sys.argv[3])
for w in wls:
    for v in ("main", "var"):
        ks = [json.load(open(f"gpurun_out/{tag}_{w}_{v}_{i}.json")) for i in range(1, n + 1)]
        print(w, v, "kernel ms", [d["kernels"][d["roofline"]["kernel"]]["ms_per_launch"] for d in ks],
              "step ms", [d["ms_per_step"] for d in ks], "rounds", [d["rounds_per_step"] for d in ks])
PY
