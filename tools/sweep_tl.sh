set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_timeline_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/tl6.log 2>&1 || { tail -30 gpurun_out/tl6.log; exit 1; }
tail -2 gpurun_out/tl6.log
for sl in 4 16 32; do
  FIT_TL_SLICES=$sl timeout -k 10 200 python -u bench.py --workload c5 --steps 3 --warmup 1 --no-cpu > gpurun_out/c5_sl$sl.json 2>/dev/null || exit 1
  python -c "import json;d=json.load(open('gpurun_out/c5_sl$sl.json'));print($sl, d['value'], d['ms_per_step'], d['kernels'])"
done
timeout -k 10 200 python -u tools/tl_stamps.py > gpurun_out/tl_stamps7.txt 2>&1; cat gpurun_out/tl_stamps7.txt
