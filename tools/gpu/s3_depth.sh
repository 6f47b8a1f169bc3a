# bf16x3 SYRK producer ring depth A/B (libraries built with -DKFAC_S3_DEPTH=2/4/5 next
# to the default 3): wide line (default selection) and MLP with KFAC_SYRK3=1
set -o pipefail
mkdir -p gpurun_out/s3d
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], 'frac %.3f'%d['roofline']['frac'])"; }
for D in 3 2 4 5; do
  L=$PWD/bnn_kfac_amd/libkfac_hip_d$D.so; [ $D = 3 ] && L=$PWD/bnn_kfac_amd/libkfac_hip.so
  BNN_KFAC_AMD_LIB=$L timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e --no-serial > gpurun_out/s3d/wide_d$D.log 2>&1 || exit 1
  show gpurun_out/s3d/wide_d$D.log
  BNN_KFAC_AMD_LIB=$L KFAC_SYRK3=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --no-serial > gpurun_out/s3d/mlp_d$D.log 2>&1 || exit 1
  show gpurun_out/s3d/mlp_d$D.log
done
