#!/bin/bash
# acquire-free first tiles (k_engine, k_engine_tl) and conditional TL round-start release:
# parity (full suite) + interleaved A/B vs the previous commit's build
set -o pipefail
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_full.sh ${TAG} || exit 1
bash tools/gpu_abx.sh ${TAG} "c3 c2 c5" 3 head main
