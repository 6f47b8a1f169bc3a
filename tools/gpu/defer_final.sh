# records-held cap A/B (KFAC.defer_bytes 256 MiB default vs 1 GiB) on the MLP and
# LeNet-5 lines, then the round-end check of the tree
set -o pipefail
mkdir -p gpurun_out/df
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], r['kernel'], 'launches', r['launches'], 'avg_us %.1f'%r['avg_launch_us'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/df/mlp_d_$r.log 2>&1 || exit 1
  show gpurun_out/df/mlp_d_$r.log
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --defer-mb 1024 > gpurun_out/df/mlp_1g_$r.log 2>&1 || exit 1
  show gpurun_out/df/mlp_1g_$r.log
done
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/df/lenet_d.log 2>&1 || exit 1
show gpurun_out/df/lenet_d.log
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 --defer-mb 1024 > gpurun_out/df/lenet_1g.log 2>&1 || exit 1
show gpurun_out/df/lenet_1g.log
bash tools/gpu/final_r03.sh
