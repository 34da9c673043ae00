set -o pipefail
mkdir -p gpurun_out
T=${T:-s5}
T=$T bash tools/sweep_var.sh ${VARS:-base u128} 2>&1 | tee gpurun_out/${T}_sweep.txt
