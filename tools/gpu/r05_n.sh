# Round 5: the bench as the driver runs it (steps 20, warmup 5), C5 / C3 and the serial
# figure before the pipelined headline; twice
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05n
mkdir -p $O
for r in 1 2; do
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_driver_$r.log 2>&1 || { tail -20 $O/bench_driver_$r.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench_driver_$r.log').read().strip().splitlines()[-1])
print('$r', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['serial_images_per_s'], d['breakdown'])
for k,v in d['other_configs'].items(): print(k, v['value'], v['ms_per_step'], v['roofline']['kernel'], v['roofline']['frac'])"
done
