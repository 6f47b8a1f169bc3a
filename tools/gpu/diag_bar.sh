# 32-tile diagonal factorisation with two barriers fewer per 16-block: invert parity,
# grouped MLP inversion alone (new vs HEAD library), MLP lines (2 reps interleaved)
set -o pipefail
mkdir -p gpurun_out/db
timeout -k 10 300 python -u -m pytest tests/test_gpu_invert.py tests/test_gpu_golden_r02.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/db/tests.log 2>&1 || { tail -40 gpurun_out/db/tests.log; exit 1; }
tail -1 gpurun_out/db/tests.log
for L in new head; do
  if [ $L = head ]; then export BNN_KFAC_AMD_LIB=$PWD/ab_libs/libkfac_head.so; else unset BNN_KFAC_AMD_LIB; fi
  echo "$L: $(timeout -k 10 120 python tools/probe_pair.py 300)" || exit 1
done
unset BNN_KFAC_AMD_LIB
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], 'avg_us %.1f'%r['avg_launch_us'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/db/mlp_new_$r.log 2>&1 || exit 1
  show gpurun_out/db/mlp_new_$r.log
  BNN_KFAC_AMD_LIB=$PWD/ab_libs/libkfac_head.so timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/db/mlp_head_$r.log 2>&1 || exit 1
  show gpurun_out/db/mlp_head_$r.log
done
