set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_factors.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_factors.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL|Mismatch|Max" gpurun_out/gpu_factors.log | head -30; exit $rc; }
timeout -k 10 300 python bench.py --config lenet --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/bench_lenet.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench_lenet.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['breakdown'])"
bash tools/gpu/trace_lenet.sh && python - <<'PY'
import csv
rows=list(csv.DictReader(open('gpurun_out/trace_lenet/run_kernel_stats.csv')))
for r in rows[:8]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1),'us')
PY
