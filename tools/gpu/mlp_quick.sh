set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_factors.log 2>&1; rc=$?
tail -1 gpurun_out/gpu_factors.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/gpu_factors.log | head -20; exit $rc; }
for i in 1 2; do
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(round(d['value']/1e6,2), 'M img/s', round(d['ms_per_step'],4), 'ms', {k: round(v,4) for k,v in d['breakdown'].items()})"
done
