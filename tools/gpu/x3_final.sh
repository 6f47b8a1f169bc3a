# direct-load x3 (cleaned): whole GPU suite + smoke, x3-forced factor tests, MLP line
# (2 reps), LeNet-5 with x3 forced on its n <= 401 groups vs default, wide line
set -o pipefail
mkdir -p gpurun_out/x3z
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/x3z/tests.log 2>&1 || { tail -40 gpurun_out/x3z/tests.log; exit 1; }
tail -1 gpurun_out/x3z/tests.log
KFAC_TILES_X3=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py tests/test_gpu_invert.py tests/test_gpu_golden_r02.py tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/x3z/tests_forced.log 2>&1 || { tail -40 gpurun_out/x3z/tests_forced.log; exit 1; }
tail -1 gpurun_out/x3z/tests_forced.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/x3z/smoke.log 2>&1 || { tail -20 gpurun_out/x3z/smoke.log; exit 1; }
tail -1 gpurun_out/x3z/smoke.log
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], r['kernel'], 'avg_us %.1f'%r['avg_launch_us'], 'frac %.3f'%r['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/x3z/mlp_$r.log 2>&1 || exit 1
  show gpurun_out/x3z/mlp_$r.log
done
for V in 1 d; do
  E=""; [ $V = 1 ] && E="KFAC_TILES_X3=1"
  env $E timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/x3z/lenet_$V.log 2>&1 || exit 1
  show gpurun_out/x3z/lenet_$V.log
done
timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e > gpurun_out/x3z/wide.log 2>&1 || exit 1
show gpurun_out/x3z/wide.log
