# Graph-replayed inversion steps: parity tests, then bench A/B (graph x async worker).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_invert.py tests/test_gpu_factors.py tests/test_gpu_sample.py tests/test_gpu_eig_variance.py -x -q --timeout 200 --timeout-method thread > gpurun_out/graph_tests.log 2>&1 || { tail -30 gpurun_out/graph_tests.log; exit 1; }
tail -1 gpurun_out/graph_tests.log
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'], 'serial %.3e'%(d['serial_images_per_s'] or 0))" $1; }
for rep in 1 2; do
  KFAC_INV_GRAPH=0 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/g0.log 2>&1 || exit 1; summ gpurun_out/g0.log
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/g1.log 2>&1 || exit 1; summ gpurun_out/g1.log
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --async-invert > gpurun_out/g1s.log 2>&1 || exit 1; summ gpurun_out/g1s.log
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --async-invert --launch-first 16 > gpurun_out/g1s16.log 2>&1 || exit 1; summ gpurun_out/g1s16.log
done
