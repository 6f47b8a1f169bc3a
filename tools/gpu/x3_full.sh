# x3 default: the whole GPU suite + smoke, LeNet-5 line x3 vs fp32, wide line
set -o pipefail
mkdir -p gpurun_out/x3f
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/x3f/tests.log 2>&1 || { tail -40 gpurun_out/x3f/tests.log; exit 1; }
tail -1 gpurun_out/x3f/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/x3f/smoke.log 2>&1 || { tail -20 gpurun_out/x3f/smoke.log; exit 1; }
tail -1 gpurun_out/x3f/smoke.log
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], r['kernel'], 'avg_us %.1f'%r['avg_launch_us'], 'frac %.3f'%r['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for V in 1 0; do
  KFAC_TILES_X3=$V timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/x3f/lenet_$V.log 2>&1 || exit 1
  show gpurun_out/x3f/lenet_$V.log
done
timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e > gpurun_out/x3f/wide.log 2>&1 || exit 1
show gpurun_out/x3f/wide.log
