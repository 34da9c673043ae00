set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
T=${1:-r02i}
for v in stamps st_notie st_idle4; do
  timeout -k 10 120 python -u tools/mw_stamps.py c3 libfitgpu_$v.so > gpurun_out/${T}_$v.txt 2>&1 || { tail gpurun_out/${T}_$v.txt; exit 1; }
  echo "== $v"; head -4 gpurun_out/${T}_$v.txt
done
