#!/bin/bash
# Round 6: class engine (k_class) A/Bs — its GPU tests, a paired A/B of the current build against a
# variant library ($2, default fitgpu/libfitgpu_clsold.so) with FIT_ENGINE=class on C4 / C3 / C2,
# the default engine choice beside it, and the stamps build's per-segment cycles.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06w}
VAR=${2:-slurm-bridge-operator_amd/fitgpu/libfitgpu_clsold.so}
timeout -k 10 600 python -u -m pytest tests/test_class_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/${T}_tests.txt 2>&1 || { tail -30 gpurun_out/${T}_tests.txt; exit 1; }
tail -1 gpurun_out/${T}_tests.txt
Q="--no-cpu --no-live-pmc --no-shard-price --no-device-path --steps 5 --warmup 2 --repeats 1"
for i in 1 2; do
  for w in c4 c3 c2; do
    FIT_ENGINE=class timeout -k 10 300 python -u bench.py --workload $w $Q > gpurun_out/${T}_${w}_new_$i.json 2> gpurun_out/${T}_${w}_new_$i.err || { tail -5 gpurun_out/${T}_${w}_new_$i.err; exit 1; }
    FIT_ENGINE=class FITGPU_LIB=$VAR timeout -k 10 300 python -u bench.py --workload $w $Q > gpurun_out/${T}_${w}_old_$i.json 2> gpurun_out/${T}_${w}_old_$i.err || { tail -5 gpurun_out/${T}_${w}_old_$i.err; exit 1; }
  done
done
for w in c4 c3; do
  timeout -k 10 300 python -u bench.py --workload $w $Q > gpurun_out/${T}_${w}_persistent.json 2> gpurun_out/${T}_${w}_persistent.err || { tail -5 gpurun_out/${T}_${w}_persistent.err; exit 1; }
done
python3 - "$T" <<'PY'
import json, sys
t = sys.argv[1]
def k(f):
    d = json.load(open(f)); r = d["roofline"]["kernel"]; return round(d["kernels"][r]["ms_per_launch"], 2), r
for w in ("c4", "c3", "c2"):
    print(w, "new", [k(f"gpurun_out/{t}_{w}_new_{i}.json") for i in (1, 2)], "old", [k(f"gpurun_out/{t}_{w}_old_{i}.json") for i in (1, 2)])
for w in ("c4", "c3"):
    print(w, "persistent", k(f"gpurun_out/{t}_{w}_persistent.json"))
PY
for w in c4 c3; do timeout -k 10 300 python -u tools/cls_stamps.py $w > gpurun_out/${T}_${w}_stamps.txt 2>&1 || { tail -5 gpurun_out/${T}_${w}_stamps.txt; exit 1; }; head -9 gpurun_out/${T}_${w}_stamps.txt; done
