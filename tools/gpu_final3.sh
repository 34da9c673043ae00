set -o pipefail
TAG=${1:-r04g}
bash tools/gpu_final.sh ${TAG:-r04g} || exit 1
FITGPU_STAMPS_LIB=$PWD/slurm-bridge-operator_amd/fitgpu/libfitgpu_tlfine.so timeout -k 10 300 python -u tools/tl_stamps.py > gpurun_out/${TAG:-r04g}_c5_tlfine.txt 2>&1 || { tail -20 gpurun_out/${TAG:-r04g}_c5_tlfine.txt; exit 1; }
grep -v "comp " gpurun_out/${TAG:-r04g}_c5_tlfine.txt
