# Round 5: LeNet-5 images per conv task above the planner's choice (KFAC_CONV_K 8 .. 64)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bj
mkdir -p $O
show() {
  python3 -c "
import json;d=json.loads(open('$O/$1.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$1', d['value'], round(d['ms_per_step'],4), 'factor', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4))"
}
B="python3 bench.py --config lenet --steps 50 --warmup 5 --no-cpu-baseline --no-e2e --no-serial"
for r in 1 2; do
timeout -k 10 200 $B > $O/def_$r.log 2>&1 && show def_$r || exit 1
for k in 8 16 32 64; do
KFAC_CONV_K=$k timeout -k 10 200 $B > $O/k${k}_$r.log 2>&1 && show k${k}_$r || exit 1
done
done
