set -o pipefail
export TMPDIR=/tmp
Q="--no-cpu --no-live-pmc --no-shard-price --no-device-path"
for i in 1 2; do
  timeout -k 10 300 python -u bench.py $Q > gpurun_out/r05j_main_$i.json 2>/dev/null || exit 1
  FIT_REC_BACKUP=0 timeout -k 10 300 python -u bench.py $Q > gpurun_out/r05j_nobak_$i.json 2>/dev/null || exit 1
  FITGPU_LIB=abroot/libfitgpu_r4.so timeout -k 10 300 python -u bench.py $Q > gpurun_out/r05j_r4_$i.json 2>/dev/null || exit 1
done
python3 -c "
import json
for v in ('main','nobak','r4'):
    print(v, [json.load(open(f'gpurun_out/r05j_{v}_{i}.json'))['kernels']['k_engine']['ms_per_launch'] for i in (1,2)])
"
