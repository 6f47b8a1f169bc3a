# pre-split bf16x3 SYRK (now the default for n >= 2048): ring slots x resident
# workgroups per CU on the wide line, v1 for reference; then the wide tests
set -o pipefail
mkdir -p gpurun_out/s3dw
timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/s3dw/tests.log 2>&1 || { tail -40 gpurun_out/s3dw/tests.log; exit 1; }
tail -1 gpurun_out/s3dw/tests.log
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], 'frac %.3f'%d['roofline']['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for L in s2w3 s2w2 s3w2 v1; do
  LIB=$PWD/bnn_kfac_amd/libkfac_hip_$L.so; [ $L = s2w3 ] || [ $L = v1 ] && LIB=$PWD/bnn_kfac_amd/libkfac_hip.so
  E=2; [ $L = v1 ] && E=1
  BNN_KFAC_AMD_LIB=$LIB KFAC_SYRK3=$E timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/s3dw/wide_$L.log 2>&1 || exit 1
  show gpurun_out/s3dw/wide_$L.log
done
