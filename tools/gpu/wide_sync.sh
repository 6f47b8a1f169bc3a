set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'])" $1; }
timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e --no-serial > gpurun_out/ws.log 2>&1 || exit 1; summ gpurun_out/ws.log
timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e --no-serial --async-invert > gpurun_out/wa.log 2>&1 || exit 1; summ gpurun_out/wa.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-serial > gpurun_out/ms.log 2>&1 || exit 1; summ gpurun_out/ms.log
