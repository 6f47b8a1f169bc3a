# fp32 SYRK planner occupancy (workgroups per CU the split plan targets): 4 (default) vs 5 vs 3
set -o pipefail
mkdir -p gpurun_out/twgs
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], 'frac %.3f'%d['roofline']['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for r in 1 2; do
for L in t4 t5 t3; do
  LIB=$PWD/bnn_kfac_amd/libkfac_hip_$L.so; [ $L = t4 ] && LIB=$PWD/bnn_kfac_amd/libkfac_hip.so
  BNN_KFAC_AMD_LIB=$LIB timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/twgs/mlp_${L}_$r.log 2>&1 || exit 1
  show gpurun_out/twgs/mlp_${L}_$r.log
done
done
BNN_KFAC_AMD_LIB=$PWD/bnn_kfac_amd/libkfac_hip_t5.so timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/twgs/lenet_t5.log 2>&1 || exit 1
show gpurun_out/twgs/lenet_t5.log
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/twgs/lenet_t4.log 2>&1 || exit 1
show gpurun_out/twgs/lenet_t4.log
