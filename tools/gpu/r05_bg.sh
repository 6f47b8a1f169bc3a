# Round 5: hardware queues per process (GPU_MAX_HW_QUEUES, HIP's default 4 on this pool)
# 4 vs 8 for the MLP line (100 steps) and LeNet-5, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bg
mkdir -p $O
run() {
  tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python3 bench.py --config $cfg --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs --no-serial > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$tag', d['value'], round(d['ms_per_step'],4), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4), 'host', round(b['host_issue_ms_per_step'],4))"
}
for r in 1 2; do
run q4_$r mlp GPU_MAX_HW_QUEUES=4
run q8_$r mlp GPU_MAX_HW_QUEUES=8
done
run l_q4 lenet GPU_MAX_HW_QUEUES=4
run l_q8 lenet GPU_MAX_HW_QUEUES=8
