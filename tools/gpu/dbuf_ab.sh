# Double-buffered packed factors: overlap/distributed parity tests, then bench A/B.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_invert.py tests/test_gpu_distributed.py tests/test_gpu_golden_r02.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dbuf_tests.log 2>&1 || { tail -30 gpurun_out/dbuf_tests.log; exit 1; }
tail -1 gpurun_out/dbuf_tests.log
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'])" $1; }
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --no-serial --single-buffer > gpurun_out/d0.log 2>&1 || exit 1; summ gpurun_out/d0.log
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --no-serial > gpurun_out/d1.log 2>&1 || exit 1; summ gpurun_out/d1.log
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --no-serial --launch-first 16 > gpurun_out/d16.log 2>&1 || exit 1; summ gpurun_out/d16.log
done
timeout -k 10 200 python bench.py --config wide --no-cpu-baseline --no-e2e --no-serial > gpurun_out/dw.log 2>&1 || exit 1; summ gpurun_out/dw.log
