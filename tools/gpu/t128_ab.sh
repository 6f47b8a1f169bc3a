# 128x128 fp32 SYRK (KFAC_T128=1): parity with every row-major group through it, then
# MLP A/B against the 64x64 kernel and the wide line against the bf16x3 default.
set -o pipefail
mkdir -p gpurun_out/t128
KFAC_T128=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/t128/tests.log 2>&1 || { tail -40 gpurun_out/t128/tests.log; exit 1; }
tail -1 gpurun_out/t128/tests.log
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], d['roofline']['kernel'], 'frac %.3f'%d['roofline']['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for r in 1 2; do
for T in 1 0; do
  KFAC_T128=$T timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/t128/mlp_${T}_$r.log 2>&1 || exit 1
  show gpurun_out/t128/mlp_${T}_$r.log
done
done
KFAC_T128=1 KFAC_SYRK3=0 timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e > gpurun_out/t128/wide_t128.log 2>&1 || exit 1
show gpurun_out/t128/wide_t128.log
