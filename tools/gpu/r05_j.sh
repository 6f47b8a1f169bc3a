# Round 5: the pass's deferred reduce on the inversion side stream (KFAC.reduce_on_side):
# parity tests, same-process A/B, the second-KFAC probe, the bench line (with C3 / C5),
# the step timeline and the PMC passes of the bench's kernels
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05j
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_c2.py tests/test_gpu_ragged.py tests/test_gpu_invert.py tests/test_gpu_factors.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 200 python tools/probe_side_reduce.py mlp 300 3 > $O/ab_mlp.log 2>&1 || { tail -20 $O/ab_mlp.log; exit 1; }
tail -1 $O/ab_mlp.log
timeout -k 10 200 python tools/probe_side_reduce.py lenet 30 2 > $O/ab_lenet.log 2>&1 || { tail -20 $O/ab_lenet.log; exit 1; }
tail -1 $O/ab_lenet.log
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
