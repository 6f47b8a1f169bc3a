# Round 4: cached fast-path templates across cycles (GPU suite, smoke, bench + host profile)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04l
mkdir -p $O
summ() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2], round(d['value']/1e6,2),'M img/s', round(d['ms_per_step'],4),'ms', round(r['avg_launch_us'],1),'us', round(r['frac'],3), d['breakdown'].get('host_issue_ms_per_step'), d.get('serial_images_per_s'))" "$@"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 200 python tools/host_api_bench.py 200 > $O/host_api.log 2>&1 || { tail -20 $O/host_api.log; exit 1; }
echo "host api: $(tail -1 $O/host_api.log)"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --host-profile $O/host_profile.txt > $O/bench_mlp.log 2>&1 || { tail -20 $O/bench_mlp.log; exit 1; }
summ $O/bench_mlp.log default
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > $O/bench_mlp2.log 2>&1 || { tail -20 $O/bench_mlp2.log; exit 1; }
summ $O/bench_mlp2.log default2
head -24 $O/host_profile.txt
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --no-serial > $O/bench_lenet.log 2>&1 || { tail -20 $O/bench_lenet.log; exit 1; }
summ $O/bench_lenet.log lenet
