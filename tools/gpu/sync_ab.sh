# Async-worker vs in-thread phase 1 of the inversion (graph replay makes it one call).
set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'])" $1; }
for rep in 1 2 3; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --no-serial --async-invert > gpurun_out/sa.log 2>&1 || exit 1; summ gpurun_out/sa.log
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --no-serial > gpurun_out/ss.log 2>&1 || exit 1; summ gpurun_out/ss.log
done
timeout -k 10 200 python tools/host_probe.py > gpurun_out/hs.log 2>&1; grep -v amdgpu gpurun_out/hs.log | tail -3
