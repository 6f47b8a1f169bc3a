# First-launch size A/B on the MLP line (KFAC.launch_first; doubling afterwards),
# pipelined and serial (pass, then invert) rates.
set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'serial %.3e'%(d['serial_images_per_s'] or 0), 'ms/step %.3f'%d['ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'])" $1; }
for rep in 1 2; do
  for lf in 1 4 6 8 16; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --launch-first $lf > gpurun_out/lf$lf.log 2>&1 || exit 1; summ gpurun_out/lf$lf.log
  done
done
