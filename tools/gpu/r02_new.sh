# Round-2 additions on the GPU: new test files, the full suite, then the bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_distributed.py tests/test_gpu_golden_r02.py tests/test_gpu_wide.py -x -v --timeout 200 --timeout-method thread > gpurun_out/new_tests.log 2>&1 || { tail -60 gpurun_out/new_tests.log; exit 1; }
tail -3 gpurun_out/new_tests.log
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1 || { tail -40 gpurun_out/gpu_tests.log; exit 1; }
tail -2 gpurun_out/gpu_tests.log
timeout -k 10 300 python bench.py > gpurun_out/bench_mlp.log 2>&1 || { tail -20 gpurun_out/bench_mlp.log; exit 1; }
tail -1 gpurun_out/bench_mlp.log | cut -c1-400
timeout -k 10 300 python bench.py --gpus 2 > gpurun_out/bench_gpus2.log 2>&1; echo "gpus2 rc=$?"; tail -2 gpurun_out/bench_gpus2.log
