# full GPU suite + smoke on the current tree, LeNet-5 line + kernel trace (the
# channel_small 32-bit index change), MLP line
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/c2
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/c2/tests.log 2>&1 || { tail -40 gpurun_out/c2/tests.log; exit 1; }
tail -1 gpurun_out/c2/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/c2/smoke.log 2>&1 || { tail -20 gpurun_out/c2/smoke.log; exit 1; }
tail -1 gpurun_out/c2/smoke.log
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], r['kernel'], 'avg_us %.1f'%r['avg_launch_us'], 'frac %.3f'%r['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/c2/lenet.log 2>&1 || exit 1
show gpurun_out/c2/lenet.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/c2/trace_lenet -o run -- python3 bench.py --config lenet --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/c2/trace_lenet.log 2>&1 || exit 1
head -8 gpurun_out/c2/trace_lenet/run_kernel_stats.csv | cut -c1-150
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/c2/mlp.log 2>&1 || exit 1
show gpurun_out/c2/mlp.log
