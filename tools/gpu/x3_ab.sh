# bf16x3 SYRK with fp32 panels split in registers (kfac_factor_tiles_x3): parity with
# every row-major group forced through it, then the MLP line x3 vs fp32 (2 reps)
set -o pipefail
mkdir -p gpurun_out/x3
KFAC_TILES_X3=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py tests/test_gpu_invert.py tests/test_gpu_golden_r02.py tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/x3/tests.log 2>&1 || { tail -40 gpurun_out/x3/tests.log; exit 1; }
tail -1 gpurun_out/x3/tests.log
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], r['kernel'], 'avg_us %.1f'%r['avg_launch_us'], 'frac %.3f'%r['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for r in 1 2; do
for V in 1 0; do
  KFAC_TILES_X3=$V timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/x3/mlp_${V}_$r.log 2>&1 || exit 1
  show gpurun_out/x3/mlp_${V}_$r.log
done
done
export TMPDIR=/tmp
KFAC_TILES_X3=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/x3/prof -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/x3/prof.log 2>&1 || exit 1
python tools/kstats.py gpurun_out/x3/prof > gpurun_out/x3/kstats.txt; head -8 gpurun_out/x3/kstats.txt
