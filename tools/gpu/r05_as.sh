# Round 5: re-tune of the x3 thin-row pair knobs at inversion priority 0 (MLP, 100 steps,
# 2 alternating reps): KFAC_X3_PAIR_XS (extra pair K-splits, default 5) and KFAC_X3_PAIR
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05as
mkdir -p $O
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs --no-serial > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$tag', round(d['value']/1e8,4), round(d['ms_per_step'],4), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4))"
}
for r in 1 2; do
run xs5_$r KFAC_NONE=1
run xs3_$r KFAC_X3_PAIR_XS=3
run xs8_$r KFAC_X3_PAIR_XS=8
run xs0_$r KFAC_X3_PAIR_XS=0
run nopair_$r KFAC_X3_PAIR=0
done
