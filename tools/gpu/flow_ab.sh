# Bench A/B: dataflow inversion (one persistent launch: 2 host launches per invert) vs per-step launches.
set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'], 'serial %.3e'%(d['serial_images_per_s'] or 0))" $1; }
for rep in 1 2; do
for F in 0 1; do
for LF in 1 16; do
  KFAC_INV_FLOW=$F timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --launch-first $LF > gpurun_out/f${F}_lf$LF.log 2>&1 || exit 1
  summ gpurun_out/f${F}_lf$LF.log
done
done
done
for W in 32 128; do
  KFAC_INV_FLOW=1 KFAC_INV_FLOW_WGS=$W timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --launch-first 1 > gpurun_out/fw$W.log 2>&1 || exit 1
  summ gpurun_out/fw$W.log
done
