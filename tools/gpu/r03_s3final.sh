# bf16x3 SYRK (split pass + DMA-fed SYRK, the n >= 2048 default): parity with every
# row-major group forced through it, the wide line, and the wide profile (trace + PMC)
set -o pipefail
mkdir -p gpurun_out/r03s
KFAC_SYRK3=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py tests/test_gpu_wide.py tests/test_gpu_invert.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03s/tests.log 2>&1 || { tail -40 gpurun_out/r03s/tests.log; exit 1; }
tail -1 gpurun_out/r03s/tests.log
timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e > gpurun_out/r03s/bench_wide.log 2>&1 || exit 1
tail -1 gpurun_out/r03s/bench_wide.log | cut -c1-160
BENCH="python3 bench.py --config wide --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-serial" bash profiles/collect.sh r03_wide
