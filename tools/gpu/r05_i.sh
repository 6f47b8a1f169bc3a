# Round 5: shared inversion side streams -- the second-KFAC-in-a-process probe and the
# bench line with its C3 / C5 legs
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05i
mkdir -p $O
timeout -k 10 200 python tools/other_probe.py twice > $O/probe.log 2>&1 || { tail -20 $O/probe.log; exit 1; }
tail -1 $O/probe.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-e2e > $O/bench_mlp.log 2>&1 || { tail -20 $O/bench_mlp.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench_mlp.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['serial_images_per_s'], d['breakdown'])
for k,v in d['other_configs'].items(): print(k, v['value'], v['ms_per_step'], v['roofline']['kernel'], v['roofline']['frac'], v['breakdown'])"
timeout -k 10 150 python tools/step_timeline.py 60 > $O/timeline.log 2>&1 || { tail -20 $O/timeline.log; exit 1; }
tail -1 $O/timeline.log
bash profiles/collect.sh r05pmc > $O/collect.log 2>&1 || { tail -20 $O/collect.log; exit 1; }
tail -8 $O/collect.log
