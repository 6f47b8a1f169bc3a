# Round 5: same box, the bench at the driver's step counts with and without the e2e leg
# ahead of the headline (alternating, twice each)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05p
mkdir -p $O
for r in 1 2; do
for v in e2e noe2e; do
F=""; [ $v = noe2e ] && F="--no-e2e"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $F > $O/bench_${v}_$r.log 2>&1 || { tail -20 $O/bench_${v}_$r.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench_${v}_$r.log').read().strip().splitlines()[-1])
print('$v $r', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['serial_images_per_s'])"
done
done
