# Round 5: is the cold-start ramp of the MLP step the GPU's clocks?  The warm-up probe
# after 0.3 s of unrelated GEMMs; the bench with its C5 / C3 legs first (default) at the
# driver's step counts
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05l
mkdir -p $O
timeout -k 10 200 python tools/probe_warm.py 5 20 6 0.3 > $O/warm_pre.log 2>&1 || { tail -20 $O/warm_pre.log; exit 1; }
grep block $O/warm_pre.log
timeout -k 10 400 python bench.py --steps 20 --warmup 5 > $O/bench_driver.log 2>&1 || { tail -20 $O/bench_driver.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench_driver.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['serial_images_per_s'], d['breakdown'])
for k,v in d['other_configs'].items(): print(k, v['value'], v['ms_per_step'], v['roofline']['kernel'], v['roofline']['frac'])
print(d['cpu_baseline'])"
