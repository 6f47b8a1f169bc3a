# Round 5: the pair units' extra K-split divisor (KFAC_X3_PAIR_XS) re-checked on the
# final tree (inversion pairs, prio 0): 5 (default) vs 4 vs 7
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bt
mkdir -p $O
for r in 1 2 3; do
for xs in 5 4 7; do
  KFAC_X3_PAIR_XS=$xs timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs --no-serial > $O/b_xs${xs}_$r.log 2>&1 || { tail -20 $O/b_xs${xs}_$r.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/b_xs${xs}_$r.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('xs$xs $r', d['value'], round(d['ms_per_step'],4), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4))"
done
done
