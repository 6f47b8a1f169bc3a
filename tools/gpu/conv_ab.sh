# LeNet line, same box: current tree vs the previous conv kernel build (libkfac_hip_prev.so)
set -o pipefail
mkdir -p gpurun_out/cab
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'frac %.3f'%d['roofline']['frac'])"; }
for r in 1 2; do
for L in cur prev; do
  LIB=$PWD/bnn_kfac_amd/libkfac_hip.so; [ $L = prev ] && LIB=$PWD/bnn_kfac_amd/libkfac_hip_prev.so
  BNN_KFAC_AMD_LIB=$LIB timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --no-serial --steps 20 > gpurun_out/cab/lenet_${L}_$r.log 2>&1 || exit 1
  show gpurun_out/cab/lenet_${L}_$r.log
done
done
