# bench defaults after the pipelined loop's launch_first 16: MLP (2 reps, with the CPU
# legs once), LeNet-5, wide; the same three with --launch-first 1 for reference
set -o pipefail
mkdir -p gpurun_out/lf
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], r['kernel'], 'avg_us %.1f'%r['avg_launch_us'], 'frac %.3f'%r['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0), d['config'].get('launch_first'))"; }
timeout -k 10 500 python bench.py > gpurun_out/lf/mlp_1.log 2>&1 || exit 1
show gpurun_out/lf/mlp_1.log
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/lf/mlp_2.log 2>&1 || exit 1
show gpurun_out/lf/mlp_2.log
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --launch-first 1 > gpurun_out/lf/mlp_lf1.log 2>&1 || exit 1
show gpurun_out/lf/mlp_lf1.log
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e > gpurun_out/lf/lenet.log 2>&1 || exit 1
show gpurun_out/lf/lenet.log
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --launch-first 1 > gpurun_out/lf/lenet_lf1.log 2>&1 || exit 1
show gpurun_out/lf/lenet_lf1.log
timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e > gpurun_out/lf/wide.log 2>&1 || exit 1
show gpurun_out/lf/wide.log
