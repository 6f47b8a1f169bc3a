# MLP line: bf16x3 SYRK vs fp32 64x64 kernel at first-launch sizes 1 / 4 / 16
set -o pipefail
mkdir -p gpurun_out/s3lf
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], 'launches', d['roofline']['launches'], 'host %.3f'%b['host_issue_ms_per_step'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for LF in 1 4 16; do
for S in 1 0; do
  KFAC_SYRK3=$S timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --launch-first $LF > gpurun_out/s3lf/mlp_s${S}_lf$LF.log 2>&1 || exit 1
  show gpurun_out/s3lf/mlp_s${S}_lf$LF.log
done
done
