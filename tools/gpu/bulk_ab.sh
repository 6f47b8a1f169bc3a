# Wide inversion: parity tests, wide bench line, kernel breakdown of the last inversion.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_invert.py tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread > gpurun_out/inv_tests.log 2>&1 || { tail -30 gpurun_out/inv_tests.log; exit 1; }
tail -1 gpurun_out/inv_tests.log
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'], 'serial %.3e'%(d['serial_images_per_s'] or 0))" $1; }
timeout -k 10 300 python bench.py --config wide --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/wide_bulk.log 2>&1 || exit 1
summ gpurun_out/wide_bulk.log
bash tools/gpu/wide_prof.sh
