# SYRK microbench (t64 / macro / macro grouped) + bench A/B of the launch schedule.
set -o pipefail
mkdir -p gpurun_out
(cd tools/microbench && timeout -k 10 120 ./syrk_ab > ../../gpurun_out/syrk_ab.log 2>&1) || exit 1
grep -v "noloop\|regops\|noDMA" gpurun_out/syrk_ab.log
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'], 'launches', r['launches'], 'launch_us %.1f'%r['avg_launch_us'], 'serial %.3e'%(d['serial_images_per_s'] or 0))" $1; }
for LF in 1 4 16 1 4 16; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --launch-first $LF > gpurun_out/mlp_lf$LF.log 2>&1 || exit 1
  summ gpurun_out/mlp_lf$LF.log
done
for M in 0 2; do
  KFAC_SYRK_MACRO=$M timeout -k 10 300 python bench.py --config wide --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/wide_m$M.log 2>&1 || exit 1
  summ gpurun_out/wide_m$M.log
done
KFAC_SYRK_GROUP=1 timeout -k 10 300 python bench.py --config wide --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/wide_g1.log 2>&1 || exit 1
summ gpurun_out/wide_g1.log
