# wide MLP (C5): the register-split x3 SYRK (no split pass) vs the split-pass syrk3
set -o pipefail
mkdir -p gpurun_out/wx3
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], r['kernel'], 'avg_us %.1f'%r['avg_launch_us'], 'frac %.3f'%r['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for r in 1 2; do
  KFAC_SYRK3=0 KFAC_TILES_X3=1 timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/wx3/wide_x3_$r.log 2>&1 || exit 1
  show gpurun_out/wx3/wide_x3_$r.log
  timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/wx3/wide_d_$r.log 2>&1 || exit 1
  show gpurun_out/wx3/wide_d_$r.log
done
