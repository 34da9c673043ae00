#!/bin/bash
# TL round start without the release when the last window wrote no global-slab list; TM_PREP
# removed: parity (full suite) + interleaved A/B on C5 vs the previous commit's build
set -o pipefail
TAG=$1
export TMPDIR=/tmp
mkdir -p gpurun_out
bash tools/gpu_full.sh ${TAG} || exit 1
bash tools/gpu_abx.sh ${TAG} "c5" 4 head main
