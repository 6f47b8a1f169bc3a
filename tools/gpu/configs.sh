set -o pipefail
timeout -k 10 600 python bench.py --config lenet --steps 5 --warmup 2 > gpurun_out/bench_lenet.log 2>&1; echo "lenet rc=$?"; tail -1 gpurun_out/bench_lenet.log | cut -c1-600
timeout -k 10 600 python bench.py --config wide --steps 3 --warmup 1 --images 16384 > gpurun_out/bench_wide.log 2>&1; echo "wide rc=$?"; tail -1 gpurun_out/bench_wide.log | cut -c1-600
