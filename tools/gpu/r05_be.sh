# Round 5: the deferred-verdict inversion on the two-launch steps replayed from a cached
# capture (KFAC_INV_SPLIT=1, default) vs the merged steps (=0): GPU suite, then the MLP
# line 100 steps x 3 alternating, then the driver's command once each
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05be
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$tag', round(d['value']/1e8,4), round(d['ms_per_step'],4), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4), 'host', round(b['host_issue_ms_per_step'],4), 'serial', round(d['serial_images_per_s']/1e7,3))"
}
for r in 1 2 3; do
run merged_$r KFAC_INV_SPLIT=0
run split_$r KFAC_INV_SPLIT=1
done
for v in 0 1; do
KFAC_INV_SPLIT=$v timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv_$v.log 2>&1 || { tail -20 $O/drv_$v.log; exit 1; }
python3 -c "
import json;d=json.loads(open('$O/drv_$v.log').read().strip().splitlines()[-1])
o=d['other_configs']
print('drv split=$v', round(d['value']/1e8,4), round(d['ms_per_step'],4), 'serial', round(d['serial_images_per_s']/1e7,3), 'C5', round(o['C5']['ms_per_step'],3), 'C3', round(o['C3']['ms_per_step'],3))"
done
