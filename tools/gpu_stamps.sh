#!/bin/bash
# diagnostic: decider / helper / round-start stamps (FIT_STAMPS build) on the given workloads
set -o pipefail
TAG=$1; shift
export TMPDIR=/tmp
mkdir -p gpurun_out
for wl in "$@"; do
  timeout -k 10 200 python -u tools/mw_stamps.py $wl libfitgpu_stamps.so > gpurun_out/${TAG}_${wl}_stamps.txt 2>&1 || { tail -20 gpurun_out/${TAG}_${wl}_stamps.txt; exit 1; }
  echo "== $wl"; grep -v "comp " gpurun_out/${TAG}_${wl}_stamps.txt
done
