#!/bin/bash
# Round 5 end: every -m gpu test and smoke(), the default C3 bench line, C5, then the profiles
# (rocprofv3 kernel traces for C3 / C5 / C4, PMC passes, C2 / C3o / C4 lines, admission).
set -o pipefail
TAG=${1:-r05z}
bash tools/gpu_final.sh $TAG || exit 1
bash tools/gpu_profile.sh $TAG || exit 1
echo ok
