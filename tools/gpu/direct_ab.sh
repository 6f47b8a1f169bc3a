# Barrier-free direct-load SYRK (KFAC_SYRK_DIRECT): factor parity tests per variant, then bench A/B.
set -o pipefail
mkdir -p gpurun_out
for d in 2 43; do
  KFAC_SYRK_DIRECT=$d timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_golden_r02.py tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/direct_tests_$d.log 2>&1 || { tail -30 gpurun_out/direct_tests_$d.log; exit 1; }
  echo "direct=$d: $(tail -1 gpurun_out/direct_tests_$d.log)"
done
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'], 'traffic', r.get('traffic'))" $1; }
for rep in 1 2; do
  for d in 0 2 43; do
    KFAC_SYRK_DIRECT=$d timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --no-serial > gpurun_out/dir_$d.log 2>&1 || exit 1; summ gpurun_out/dir_$d.log
  done
done
for d in 0 2 43; do
  KFAC_SYRK_DIRECT=$d timeout -k 10 200 python bench.py --config wide --no-cpu-baseline --no-e2e --no-serial > gpurun_out/dirw_$d.log 2>&1 || exit 1; summ gpurun_out/dirw_$d.log
done
