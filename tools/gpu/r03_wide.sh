# Round 3: default-path wide check (bf16x3 SYRK auto-selected at n >= 2048) and its
# profile (kernel trace + PMC passes) under gpurun_out/prof_r03_wide.
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03/tests_wide.log 2>&1 || { tail -40 gpurun_out/r03/tests_wide.log; exit 1; }
tail -1 gpurun_out/r03/tests_wide.log
timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e > gpurun_out/r03/bench_wide.log 2>&1 || exit 1
tail -1 gpurun_out/r03/bench_wide.log | cut -c1-200
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/r03/bench_mlp.log 2>&1 || exit 1
tail -1 gpurun_out/r03/bench_mlp.log | cut -c1-200
BENCH="python3 bench.py --config wide --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-serial" bash profiles/collect.sh r03_wide
