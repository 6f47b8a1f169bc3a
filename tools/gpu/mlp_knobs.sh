# MLP line with the x3 SYRK: inversion launch knobs (tasks per workgroup, wave
# priority) and the pass's first launch size, 2 reps interleaved
set -o pipefail
mkdir -p gpurun_out/knobs
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], 'host %.3f'%b['host_issue_ms_per_step'], 'avg_us %.1f'%r['avg_launch_us'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
run() { local tag=$1; shift; env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e $EXTRA > gpurun_out/knobs/$tag.log 2>&1 || exit 1; show gpurun_out/knobs/$tag.log; }
for r in 1 2; do
  EXTRA= run d_$r KFAC_NONE=1
  EXTRA= run tpw1_$r KFAC_INV_TPW=1
  EXTRA= run prio0_$r KFAC_INV_PRIO=0
  EXTRA="--launch-first 4" run lf4_$r KFAC_NONE=1
  EXTRA="--launch-first 16" run lf16_$r KFAC_NONE=1
done
