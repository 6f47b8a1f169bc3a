# x3 SYRK: direct buffer loads into registers (default build) vs the per-wave LDS-DMA
# rings (libkfac_hip_x3w.so); parity of the default first
set -o pipefail
mkdir -p gpurun_out/x3d
KFAC_TILES_X3=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py tests/test_gpu_invert.py tests/test_gpu_golden_r02.py tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/x3d/tests.log 2>&1 || { tail -40 gpurun_out/x3d/tests.log; exit 1; }
tail -1 gpurun_out/x3d/tests.log
for R in 16384 32768; do
  for L in kfac_hip kfac_hip_x3w; do
    BNN_KFAC_AMD_LIB=$PWD/bnn_kfac_amd/lib$L.so timeout -k 10 120 python tools/x3_probe.py $R > gpurun_out/x3d/p_${L}_$R.log 2>&1 || { tail -20 gpurun_out/x3d/p_${L}_$R.log; exit 1; }
    grep "x3:" gpurun_out/x3d/p_${L}_$R.log
  done
done
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], r['kernel'], 'avg_us %.1f'%r['avg_launch_us'], 'frac %.3f'%r['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for r in 1 2; do
for L in kfac_hip kfac_hip_x3w; do
  BNN_KFAC_AMD_LIB=$PWD/bnn_kfac_amd/lib$L.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/x3d/mlp_${L}_$r.log 2>&1 || exit 1
  show gpurun_out/x3d/mlp_${L}_$r.log
done
done
