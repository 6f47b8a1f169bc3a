# Round 5: side streams 2 vs 3 and max_pending 2 vs 3, merged vs split steps (MLP, 100
# steps) and LeNet-5 -- which of the new defaults cost the pipelined line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bf
mkdir -p $O
run() {
  tag=$1; cfg=$2; mp=$3; shift; shift; shift
  env "$@" timeout -k 10 200 python3 bench.py --config $cfg --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs --no-serial --max-pending $mp > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$tag', d['value'], round(d['ms_per_step'],4), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4), 'host', round(b['host_issue_ms_per_step'],4))"
}
for r in 1 2; do
run m_s2_p2_$r mlp 2 KFAC_INV_SPLIT=0 KFAC_INV_STREAMS=2
run m_s3_p3_$r mlp 3 KFAC_INV_SPLIT=0 KFAC_INV_STREAMS=3
run m_s2_p3_$r mlp 3 KFAC_INV_SPLIT=0 KFAC_INV_STREAMS=2
run s_s3_p3_$r mlp 3 KFAC_INV_SPLIT=1 KFAC_INV_STREAMS=3
done
run l_s2_p2 lenet 2 KFAC_INV_SPLIT=0 KFAC_INV_STREAMS=2
run l_s3_p3 lenet 3 KFAC_INV_SPLIT=0 KFAC_INV_STREAMS=3
