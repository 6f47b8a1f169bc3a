# syrk3 quick check: factor parity tests, wide + MLP bench lines, PMC issue counters on wide
set -o pipefail
mkdir -p gpurun_out/s3
KFAC_SYRK3=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3/tests.log 2>&1 || { tail -40 gpurun_out/s3/tests.log; exit 1; }
tail -1 gpurun_out/s3/tests.log
KFAC_SYRK3=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/s3/mlp_1.log 2>&1 || exit 1
KFAC_SYRK3=1 timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e > gpurun_out/s3/wide_1.log 2>&1 || exit 1
bash tools/gpu/s3_pmc.sh
