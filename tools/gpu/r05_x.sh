# Round 5: the serial loop's first launch size (launch sizes then double; 15 updates per
# MLP pass): serial img/s per launch_first, one box
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05x
mkdir -p $O
for lf in 1 5 3 7 1 5; do
timeout -k 10 300 python bench.py --steps 40 --warmup 5 --launch-first $lf --no-cpu-baseline --no-e2e --no-other-configs > $O/bench_lf$lf.log 2>&1 || { tail -20 $O/bench_lf$lf.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench_lf$lf.log').read().strip().splitlines()[-1])
print('lf $lf', d['serial_images_per_s'], d['value'])"
done
