# bf16x3 SYRK on pre-split panels (KFAC_SYRK3=2): parity, then wide / MLP lines vs the
# default kernels, substep rings of 3 / 4 (default) / 6 slots
set -o pipefail
mkdir -p gpurun_out/s3d2
KFAC_SYRK3=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s3d2/tests.log 2>&1 || { tail -40 gpurun_out/s3d2/tests.log; exit 1; }
tail -1 gpurun_out/s3d2/tests.log
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], d['roofline']['kernel'], 'frac %.3f'%d['roofline']['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for L in s4 s3 s6; do
  LIB=$PWD/bnn_kfac_amd/libkfac_hip_$L.so; [ $L = s4 ] && LIB=$PWD/bnn_kfac_amd/libkfac_hip.so
  BNN_KFAC_AMD_LIB=$LIB KFAC_SYRK3=2 timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e --steps 10 > gpurun_out/s3d2/wide_2$L.log 2>&1 || exit 1
  show gpurun_out/s3d2/wide_2$L.log
done
KFAC_SYRK3=1 timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e --steps 10 > gpurun_out/s3d2/wide_1.log 2>&1 || exit 1
show gpurun_out/s3d2/wide_1.log
for V in 2 0; do
  KFAC_SYRK3=$V timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/s3d2/mlp_$V.log 2>&1 || exit 1
  show gpurun_out/s3d2/mlp_$V.log
done
