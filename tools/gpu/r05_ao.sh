# Round 5: kfac_factor_tiles_x3 planned for 1 (default) / 2 / 3 dispatch rounds on the MLP
# (KFAC_X3_ROUNDS): more, shorter tasks let the hardware dispatcher hand a CU slowed by
# the overlapped inversion fewer of them; 2 alternating reps of 100 steps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ao
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
run r1_$r KFAC_NONE=1
run r2_$r KFAC_X3_ROUNDS=2
run r3_$r KFAC_X3_ROUNDS=3
done
