# Conv SYRK changes: factor parity tests, microbench, LeNet bench line.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_golden_r02.py tests/test_gpu_invert.py -x -q --timeout 200 --timeout-method thread > gpurun_out/conv_tests.log 2>&1 || { tail -30 gpurun_out/conv_tests.log; exit 1; }
tail -1 gpurun_out/conv_tests.log
(cd tools/microbench && timeout -k 10 120 ./conv_ab > ../../gpurun_out/conv_ab.log 2>&1) || { tail gpurun_out/conv_ab.log; exit 1; }
grep "us  (" gpurun_out/conv_ab.log | cut -c1-80
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e > gpurun_out/bench_lenet2.log 2>&1 || { tail -5 gpurun_out/bench_lenet2.log; exit 1; }
python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'], 'serial %.3e'%(d['serial_images_per_s'] or 0))" gpurun_out/bench_lenet2.log
