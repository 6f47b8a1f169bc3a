# sample kernel parity + full GPU suite, then the wide bench (single side stream for
# throughput-bound inversions) and the MLP bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_sample.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_sample.log 2>&1 || { tail -40 gpurun_out/gpu_sample.log; exit 1; }
tail -3 gpurun_out/gpu_sample.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -30 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 600 python bench.py --config wide --steps 3 --warmup 1 --images 16384 > gpurun_out/bench_wide.log 2>&1 || exit $?
tail -1 gpurun_out/bench_wide.log | cut -c1-200
timeout -k 10 600 python bench.py > gpurun_out/bench_mlp.log 2>&1 || exit $?
tail -1 gpurun_out/bench_mlp.log | cut -c1-200
