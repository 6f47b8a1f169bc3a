# Round 5: the two-launch (stored panel) inversion steps beside the MLP pass at priority 0
# (timing build ab_libs/merge0 with a KFAC_INV_MERGE_T override): the SYRK's time beside
# it vs the merged steps; max_pending 3 (the longer chain)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bd
mkdir -p $O
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs --max-pending 3 > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$tag', round(d['value']/1e8,4), round(d['ms_per_step'],4), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4), 'host', round(b['host_issue_ms_per_step'],4), 'serial', round(d['serial_images_per_s']/1e7,3))"
}
for r in 1 2; do
run merged_$r BNN_KFAC_AMD_LIB=ab_libs/merge0/libkfac_hip.so
run twolaunch_$r BNN_KFAC_AMD_LIB=ab_libs/merge0/libkfac_hip.so KFAC_INV_MERGE_T=0
done
