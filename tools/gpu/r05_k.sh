# Round 5: warm-up of the pipelined MLP step (blocks of 20 timed steps from a cold
# start), the bench at the driver's step counts and at 300 steps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05k
mkdir -p $O
timeout -k 10 200 python tools/probe_warm.py 5 20 12 > $O/warm.log 2>&1 || { tail -20 $O/warm.log; exit 1; }
cat $O/warm.log | grep block
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-other-configs > $O/bench_20.log 2>&1 || { tail -20 $O/bench_20.log; exit 1; }
timeout -k 10 300 python bench.py --steps 300 --warmup 10 --no-cpu-baseline --no-e2e --no-other-configs > $O/bench_300.log 2>&1 || { tail -20 $O/bench_300.log; exit 1; }
for f in bench_20 bench_300; do python -c "
import json;d=json.loads(open('$O/$f.log').read().strip().splitlines()[-1])
print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['serial_images_per_s'], d['breakdown'])"; done
