# Round 5: inversion wave priority 3 (default) vs 0 / 2, and 0 with one task per
# workgroup, beside the MLP pass: 3 alternating reps of 100 steps, then the driver's
# command (20 steps, warmup 5, C5 / C3 legs first) at priority 3 and 0
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05am
mkdir -p $O
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$tag', round(d['value']/1e8,4), round(d['ms_per_step'],4), 'serial', round(d['serial_images_per_s']/1e7,3), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4), 'host', round(b['host_issue_ms_per_step'],4))"
}
drv() {
  tag=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1])
o=d['other_configs']
print('$tag', round(d['value']/1e8,4), round(d['ms_per_step'],4), 'serial', round(d['serial_images_per_s']/1e7,3), 'C5', round(o['C5']['ms_per_step'],3), 'C3', round(o['C3']['ms_per_step'],3))"
}
for r in 1 2 3; do
run p3_$r KFAC_INV_PRIO=3
run p0_$r KFAC_INV_PRIO=0
run p2_$r KFAC_INV_PRIO=2
run p0t1_$r KFAC_INV_PRIO=0 KFAC_INV_TPW=1
done
drv drv_p3 KFAC_INV_PRIO=3
drv drv_p0 KFAC_INV_PRIO=0
drv drv_p3b KFAC_INV_PRIO=3
drv drv_p0b KFAC_INV_PRIO=0
