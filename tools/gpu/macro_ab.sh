# A/B of the 128x128 macro-tile SYRK (KFAC_SYRK_MACRO=1, default) vs the 64-tile launch.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_wide.py tests/test_gpu_distributed.py -x -q --timeout 200 --timeout-method thread > gpurun_out/factor_tests.log 2>&1 || { tail -40 gpurun_out/factor_tests.log; exit 1; }
tail -1 gpurun_out/factor_tests.log
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'], 'launch_us %.1f'%r['avg_launch_us'], 'serial %.3e'%(d['serial_images_per_s'] or 0))" $1; }
for M in 0 1 0 1; do
  KFAC_SYRK_MACRO=$M timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/mlp_m$M.log 2>&1 || exit 1
  summ gpurun_out/mlp_m$M.log
done
for M in 0 1; do
  KFAC_SYRK_MACRO=$M timeout -k 10 300 python bench.py --config wide --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/wide_m$M.log 2>&1 || exit 1
  summ gpurun_out/wide_m$M.log
done
