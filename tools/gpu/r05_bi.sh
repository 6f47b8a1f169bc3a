# Round 5: LeNet-5 (C3) conv task sizing re-check at the 512 MiB records cap: images
# per conv task (KFAC_CONV_K; default = the planner's fill-once k), the n <= 8 channel
# kernel on/off (KFAC_CONV_SMALL), the 1 GiB records cap; 50 steps each, twice
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bi
mkdir -p $O
show() {
  python3 -c "
import json;d=json.loads(open('$O/$1.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$1', d['value'], round(d['ms_per_step'],4), 'factor', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4), 'host', round(b['host_issue_ms_per_step'],4))"
}
B="python3 bench.py --config lenet --steps 50 --warmup 5 --no-cpu-baseline --no-e2e --no-serial"
for r in 1 2; do
timeout -k 10 200 $B > $O/def_$r.log 2>&1 && show def_$r || exit 1
KFAC_CONV_K=1 timeout -k 10 200 $B > $O/k1_$r.log 2>&1 && show k1_$r || exit 1
KFAC_CONV_K=2 timeout -k 10 200 $B > $O/k2_$r.log 2>&1 && show k2_$r || exit 1
KFAC_CONV_K=4 timeout -k 10 200 $B > $O/k4_$r.log 2>&1 && show k4_$r || exit 1
KFAC_CONV_SMALL=0 timeout -k 10 200 $B > $O/small0_$r.log 2>&1 && show small0_$r || exit 1
timeout -k 10 200 $B --defer-mb 1024 > $O/defer1g_$r.log 2>&1 && show defer1g_$r || exit 1
done
