# Round 5: bench.py with 8 hardware queues (its default now: three side streams, the
# deferred-verdict inversion on the two-launch steps replayed from a capture) vs 4 (two
# side streams, merged steps): GPU suite, MLP 100 steps x 3, LeNet-5, driver command
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bh
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
run() {
  tag=$1; cfg=$2; shift; shift
  env "$@" timeout -k 10 200 python3 bench.py --config $cfg --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs --no-serial > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$tag', d['value'], round(d['ms_per_step'],4), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4), 'host', round(b['host_issue_ms_per_step'],4))"
}
for r in 1 2 3; do
run q4_$r mlp GPU_MAX_HW_QUEUES=4
run q8_$r mlp GPU_MAX_HW_QUEUES=8
done
run l_q4 lenet GPU_MAX_HW_QUEUES=4
run l_q8 lenet GPU_MAX_HW_QUEUES=8
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > $O/drv.log 2>&1 || { tail -20 $O/drv.log; exit 1; }
python3 -c "
import json;d=json.loads(open('$O/drv.log').read().strip().splitlines()[-1])
o=d['other_configs']
print('drv', round(d['value']/1e8,4), round(d['ms_per_step'],4), 'serial', round(d['serial_images_per_s']/1e7,3), 'C5', round(o['C5']['ms_per_step'],3), 'C3', round(o['C3']['ms_per_step'],3))"
