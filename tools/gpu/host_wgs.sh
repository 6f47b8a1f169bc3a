# MLP line: bench.py with per-batch record views made outside the timed loop (this
# tree) vs HEAD's bench (slices inside it), and the x3 SYRK's resident workgroups per
# CU (KFAC_X3_WGS 4 / 3 / 2)
set -o pipefail
mkdir -p gpurun_out/hw
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], r['kernel'], 'avg_us %.1f'%r['avg_launch_us'], 'frac %.3f'%r['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/hw/mlp_new_$r.log 2>&1 || exit 1
  show gpurun_out/hw/mlp_new_$r.log
  timeout -k 10 200 python bench_head.py --no-cpu-baseline --no-e2e > gpurun_out/hw/mlp_head_$r.log 2>&1 || exit 1
  show gpurun_out/hw/mlp_head_$r.log
  KFAC_X3_WGS=3 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/hw/mlp_w3_$r.log 2>&1 || exit 1
  show gpurun_out/hw/mlp_w3_$r.log
done
KFAC_X3_WGS=2 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/hw/mlp_w2.log 2>&1 || exit 1
show gpurun_out/hw/mlp_w2.log
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/hw/lenet.log 2>&1 || exit 1
show gpurun_out/hw/lenet.log
