# Round 4: ablation microbench (what bounds the bf16x3 register-split SYRK), then the
# software-pipelined kfac_factor_tiles_x3 through the GPU suite and the bench line
# (+ a host-side profile of the pipelined step in microseconds)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 120 ./tools/microbench/x3w_mb > $O/x3w_mb.log 2>&1; echo "x3w_mb rc $?"; cat $O/x3w_mb.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --host-profile $O/host_profile.txt > $O/bench_mlp.log 2>&1 || { tail -20 $O/bench_mlp.log; exit 1; }
tail -1 $O/bench_mlp.log | cut -c1-300
python -c "import json;d=json.loads(open('$O/bench_mlp.log').read().strip().splitlines()[-1]);print(json.dumps(d['roofline'])[:400]);print(d['breakdown'], d['serial_images_per_s'])"
head -50 $O/host_profile.txt
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --no-serial > $O/bench_lenet.log 2>&1 || { tail -20 $O/bench_lenet.log; exit 1; }
tail -1 $O/bench_lenet.log | cut -c1-200
timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e --no-serial > $O/bench_wide.log 2>&1 || { tail -20 $O/bench_wide.log; exit 1; }
tail -1 $O/bench_wide.log | cut -c1-200
KFAC_SYRK3=0 KFAC_TILES_X3=1 timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e --no-serial > $O/bench_wide_x3.log 2>&1 || { tail -20 $O/bench_wide_x3.log; exit 1; }
tail -1 $O/bench_wide_x3.log | cut -c1-200
