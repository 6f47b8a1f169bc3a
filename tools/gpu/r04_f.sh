# Round 4: the raw-event pipelined invert host path through the GPU suite, smoke, the
# default bench line (+ host profile) and the pipelined loop's first-launch size
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --host-profile $O/host_profile.txt > $O/bench_mlp.log 2>&1 || { tail -20 $O/bench_mlp.log; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_mlp.log').read().strip().splitlines()[-1]);r=d['roofline'];print('default', round(d['value']/1e6,2),'M img/s', round(d['ms_per_step'],4),'ms', round(r['avg_launch_us'],1),'us', round(r['frac'],3), d['breakdown'], d['serial_images_per_s'])"
head -30 $O/host_profile.txt
for lf in 4 8; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-serial --launch-first $lf > $O/bench_lf$lf.log 2>&1 || { tail -20 $O/bench_lf$lf.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_lf$lf.log').read().strip().splitlines()[-1]);r=d['roofline'];print('lf$lf', round(d['value']/1e6,2),'M img/s', round(d['ms_per_step'],4),'ms', round(r['avg_launch_us'],1),'us', round(r['frac'],3), d['breakdown']['host_issue_ms_per_step'])"
done
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --no-serial > $O/bench_lenet.log 2>&1 || { tail -20 $O/bench_lenet.log; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_lenet.log').read().strip().splitlines()[-1]);r=d['roofline'];print('lenet', round(d['value']/1e6,3),'M img/s', round(d['ms_per_step'],4),'ms', d['breakdown']['host_issue_ms_per_step'])"
