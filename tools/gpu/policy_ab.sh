# Bench A/B of the SYRK launch policy: idle-stream (default) vs doubling from 1 / 16.
set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'], 'launches', r['launches'], 'serial %.3e'%(d['serial_images_per_s'] or 0), 'e2e %.3e'%(d['e2e_images_per_s'] or 0))" $1; }
for rep in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/pol_idle.log 2>&1 || exit 1
  summ gpurun_out/pol_idle.log
  for LF in 1 16; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --launch-first $LF > gpurun_out/pol_lf$LF.log 2>&1 || exit 1
    summ gpurun_out/pol_lf$LF.log
  done
done
