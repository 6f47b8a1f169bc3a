# Round 5: stream-ordering events without the system-scope fence (KFAC._event ordering
# events; the verdict's `done` keeps it) vs every event fenced (KFAC_EVENT_FENCE=1):
# GPU suite first, then the MLP line (100 steps) and LeNet-5, alternating
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bb
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
run() {
  tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python3 bench.py --config $cfg --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs --no-serial > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$tag', d['value'], round(d['ms_per_step'],4), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4))"
}
for r in 1 2 3; do
run fence_$r mlp KFAC_EVENT_FENCE=1
run order_$r mlp KFAC_NONE=1
done
run lenet_fence lenet KFAC_EVENT_FENCE=1
run lenet_order lenet KFAC_NONE=1
