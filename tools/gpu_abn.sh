#!/bin/bash
# Paired A/B over several builds on one box (alternating): tools/gpu_abn.sh TAG WORKLOAD ROUNDS lib1 lib2 ...
# ("main" = the in-tree build); prints the k_engine ms of every run per build.
set -o pipefail
TAG=$1; W=$2; N=$3; shift 3
export TMPDIR=/tmp
mkdir -p gpurun_out
Q="--no-cpu --no-live-pmc --no-shard-price --no-device-path"
for i in $(seq 1 $N); do
  for L in "$@"; do
    n=$(basename $L .so)
    if [ "$L" = main ]; then E=""; else E="FITGPU_LIB=$L"; fi
    env $E timeout -k 10 300 python -u bench.py --workload $W $Q > gpurun_out/${TAG}_${W}_${n}_$i.json 2> gpurun_out/${TAG}_${W}_${n}_$i.err || { tail -5 gpurun_out/${TAG}_${W}_${n}_$i.err; exit 1; }
  done
done
python3 - "$TAG" "$W" "$N" "$@" <<'PY'
import json, os, sys
tag, w, n, libs = sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4:]
for L in libs:
    b = os.path.basename(L).replace(".so", "")
    ks = [json.load(open(f"gpurun_out/{tag}_{w}_{b}_{i}.json")) for i in range(1, n + 1)]
    print(f"{w} {b:18s} kernel ms", [d["kernels"][d["roofline"]["kernel"]]["ms_per_launch"] for d in ks],
          "step ms", [d["ms_per_step"] for d in ks])
PY
