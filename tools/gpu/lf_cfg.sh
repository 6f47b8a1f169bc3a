set -o pipefail
mkdir -p gpurun_out
summ() { python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'])" $1; }
for c in lenet wide; do
  for lf in 1 16; do
    timeout -k 10 300 python bench.py --config $c --no-cpu-baseline --no-e2e --no-serial --launch-first $lf > gpurun_out/lfc_${c}_$lf.log 2>&1 || exit 1; summ gpurun_out/lfc_${c}_$lf.log
  done
done
