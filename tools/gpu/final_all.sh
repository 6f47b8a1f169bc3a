# Round-end check plus the LeNet-5 (C3) and wide (C5) bench lines.
set -o pipefail
bash tools/gpu/final.sh || exit 1
timeout -k 10 300 python bench.py --config lenet > gpurun_out/bench_lenet.log 2>&1 || exit 1
tail -1 gpurun_out/bench_lenet.log | cut -c1-200
timeout -k 10 300 python bench.py --config wide --no-cpu-baseline > gpurun_out/bench_wide.log 2>&1 || exit 1
tail -1 gpurun_out/bench_wide.log | cut -c1-200
