# (1) paired-step inversion parity (KFAC_INV_PAIR=1) + the default invert suite,
# (2) MLP line pair vs default (2 reps interleaved), LeNet-5 / wide with pairs,
# (3) LeNet-5 with the x3 SYRK forced on its fully connected groups
set -o pipefail
mkdir -p gpurun_out/pair
timeout -k 10 300 python -u -m pytest tests/test_gpu_invert_pair.py tests/test_gpu_invert.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pair/tests.log 2>&1 || { tail -40 gpurun_out/pair/tests.log; exit 1; }
tail -1 gpurun_out/pair/tests.log
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], 'avg_us %.1f'%r['avg_launch_us'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
run() { local tag=$1; shift; env "$@" timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e $EXTRA > gpurun_out/pair/$tag.log 2>&1 || exit 1; show gpurun_out/pair/$tag.log; }
for r in 1 2; do
  EXTRA= run mlp_pair_$r KFAC_INV_PAIR=1
  EXTRA= run mlp_d_$r KFAC_INV_PAIR=0
done
EXTRA="--config lenet --steps 20" run lenet_pair KFAC_INV_PAIR=1
EXTRA="--config lenet --steps 20" run lenet_d KFAC_INV_PAIR=0
EXTRA="--config lenet --steps 20" run lenet_x3 KFAC_TILES_X3=1
EXTRA="--config wide" run wide_pair KFAC_INV_PAIR=1
