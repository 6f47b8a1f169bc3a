# bf16x3 staged conv (mode 0) A/B: conv parity with KFAC_CONV_X3=1, LeNet-5 lines and
# kernel traces x3 vs default
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cx3
KFAC_CONV_X3=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py tests/test_gpu_golden_r02.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/cx3/tests.log 2>&1 || { tail -40 gpurun_out/cx3/tests.log; exit 1; }
tail -1 gpurun_out/cx3/tests.log
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], r['kernel'], 'avg_us %.1f'%r['avg_launch_us'], 'frac %.3f'%r['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for r in 1 2; do
  KFAC_CONV_X3=1 timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/cx3/lenet_x3_$r.log 2>&1 || exit 1
  show gpurun_out/cx3/lenet_x3_$r.log
  timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/cx3/lenet_d_$r.log 2>&1 || exit 1
  show gpurun_out/cx3/lenet_d_$r.log
done
KFAC_CONV_X3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cx3/trace_x3 -o run -- python3 bench.py --config lenet --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/cx3/trace_x3.log 2>&1 || exit 1
head -8 gpurun_out/cx3/trace_x3/run_kernel_stats.csv | cut -c1-150
