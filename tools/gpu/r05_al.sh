# Round 5: the inversion beside the MLP pass -- wave priority, tasks per workgroup, and
# the two-launch (stored panel) steps instead of the merged ones (KFAC_INV_MERGE_T=0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05al
mkdir -p $O
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$tag', round(d['value']/1e8,4), round(d['ms_per_step'],4), 'serial', round(d['serial_images_per_s']/1e7,3), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4), 'host', round(b['host_issue_ms_per_step'],4))"
}
for r in 1 2; do
run def_$r KFAC_NONE=1
run merge0_$r KFAC_INV_MERGE_T=0
run prio0_$r KFAC_INV_PRIO=0
run prio1_$r KFAC_INV_PRIO=1
run tpw1_$r KFAC_INV_TPW=1
done
