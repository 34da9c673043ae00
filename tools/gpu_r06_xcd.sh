#!/bin/bash
# Round 6: XCD-aware task rings (fit_engine_ctl.h FIT_XCD_RINGS) — the GPU suite, then a paired
# A/B against the one-ring build (fitgpu/libfitgpu_xcd0.so) on C5 / C3 / C2, then each build's
# C5 and C3 bench line with the live PMC traffic pass.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r06x}
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${T}_gpu_tests.txt 2>&1 || { tail -40 gpurun_out/${T}_gpu_tests.txt; exit 1; }
tail -2 gpurun_out/${T}_gpu_tests.txt
bash tools/gpu_ab_r5.sh ${T}ab slurm-bridge-operator_amd/fitgpu/libfitgpu_xcd0.so "c5 c3 c2" 2 || exit 1
for w in c5 c3; do
  timeout -k 10 400 python -u bench.py --workload $w --no-cpu --no-shard-price > gpurun_out/${T}_${w}_pmc_main.json 2> gpurun_out/${T}_${w}_pmc_main.err || { tail -5 gpurun_out/${T}_${w}_pmc_main.err; exit 1; }
  FITGPU_LIB=slurm-bridge-operator_amd/fitgpu/libfitgpu_xcd0.so timeout -k 10 400 python -u bench.py --workload $w --no-cpu --no-shard-price > gpurun_out/${T}_${w}_pmc_var.json 2> gpurun_out/${T}_${w}_pmc_var.err || { tail -5 gpurun_out/${T}_${w}_pmc_var.err; exit 1; }
done
python3 - "$T" <<'PY'
import json, sys
t = sys.argv[1]
for w in ("c5", "c3"):
    for v in ("main", "var"):
        d = json.load(open(f"gpurun_out/{t}_{w}_pmc_{v}.json"))
        print(w, v, d["value"], d["ms_per_step"], d["roofline"])
PY
