# Round 4: the committed tree -- GPU suite, smoke, default bench lines (MLP x2, LeNet, wide)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04t}
mkdir -p $O
summ() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2], round(d['value']/1e6,3),'M img/s', round(d['ms_per_step'],4),'ms', round(r['avg_launch_us'],1),'us', round(r['frac'],3), d['breakdown'].get('host_issue_ms_per_step'), d.get('serial_images_per_s'))" "$@"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench_mlp.log 2>&1 || { tail -20 $O/bench_mlp.log; exit 1; }
summ $O/bench_mlp.log mlp_default
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $O/bench_mlp2.log 2>&1 || { tail -20 $O/bench_mlp2.log; exit 1; }
summ $O/bench_mlp2.log mlp_2
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e > $O/bench_lenet.log 2>&1 || { tail -20 $O/bench_lenet.log; exit 1; }
summ $O/bench_lenet.log lenet
timeout -k 10 400 python bench.py --config wide --no-cpu-baseline --no-e2e > $O/bench_wide.log 2>&1 || { tail -20 $O/bench_wide.log; exit 1; }
summ $O/bench_wide.log wide
