# MLP line: fp32 SYRK (default) vs the split-pass bf16x3 SYRK forced for every factor
set -o pipefail
mkdir -p gpurun_out/mlps3
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], d['roofline']['kernel'], 'frac %.3f'%d['roofline']['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for V in 1 0; do
  KFAC_SYRK3=$V timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/mlps3/mlp_$V.log 2>&1 || exit 1
  show gpurun_out/mlps3/mlp_$V.log
done
export TMPDIR=/tmp
KFAC_SYRK3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mlps3/prof -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/mlps3/prof.log 2>&1 || exit 1
python tools/kstats.py gpurun_out/mlps3/prof > gpurun_out/mlps3/kstats.txt; head -6 gpurun_out/mlps3/kstats.txt
