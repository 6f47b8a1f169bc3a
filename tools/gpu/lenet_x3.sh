# LeNet-5 (C3): the direct-load x3 SYRK forced on the fully connected groups
# (KFAC_TILES_X3=1, n <= 401) vs default (fp32 kfac_factor_tiles there), 2 reps
set -o pipefail
mkdir -p gpurun_out/lx3
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], r['kernel'], 'avg_us %.1f'%r['avg_launch_us'], 'frac %.3f'%r['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/lx3/lenet_d_$r.log 2>&1 || exit 1
  show gpurun_out/lx3/lenet_d_$r.log
  KFAC_TILES_X3=1 timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/lx3/lenet_x3_$r.log 2>&1 || exit 1
  show gpurun_out/lx3/lenet_x3_$r.log
done
export TMPDIR=/tmp
KFAC_TILES_X3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lx3/trace_x3 -o run -- python3 bench.py --config lenet --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/lx3/trace_x3.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/lx3/trace_d -o run -- python3 bench.py --config lenet --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/lx3/trace_d.log 2>&1 || exit 1
head -12 gpurun_out/lx3/trace_x3/run_kernel_stats.csv | cut -c1-150
head -12 gpurun_out/lx3/trace_d/run_kernel_stats.csv | cut -c1-150
