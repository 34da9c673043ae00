set -o pipefail
mkdir -p gpurun_out
T=${T:-s12}
for l in ${DECS:-}; do timeout -k 10 100 python -u tools/decbench.py $l >> gpurun_out/${T}_dec.txt 2>&1 || exit 1; done
[ -n "${DECS:-}" ] && cat gpurun_out/${T}_dec.txt
T=$T bash tools/sweep_var.sh ${VARS:-base} 2>&1 | tee gpurun_out/${T}_sweep.txt
