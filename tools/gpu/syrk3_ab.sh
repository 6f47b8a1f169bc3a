# bf16x3 SYRK (kfac_factor_syrk3) vs the fp32-MFMA kernel: parity tests, then the
# MLP and wide bench lines with KFAC_SYRK3=1 / 0, and kernel stats of the MLP line.
set -o pipefail
mkdir -p gpurun_out/s3
timeout -k 10 400 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/s3/tests.log 2>&1 || { tail -40 gpurun_out/s3/tests.log; exit 1; }
tail -2 gpurun_out/s3/tests.log
for S in 1 0; do
  KFAC_SYRK3=$S timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/s3/mlp_$S.log 2>&1 || exit 1
  tail -1 gpurun_out/s3/mlp_$S.log | cut -c1-120
done
KFAC_SYRK3=1 timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e > gpurun_out/s3/wide_1.log 2>&1 || exit 1
tail -1 gpurun_out/s3/wide_1.log | cut -c1-120
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s3/prof -o run -- python bench.py --no-cpu-baseline --no-e2e --no-serial --steps 5 > gpurun_out/s3/prof.log 2>&1 || exit 1
find gpurun_out/s3/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/s3/kernel_stats.csv
cut -d, -f1-8 gpurun_out/s3/kernel_stats.csv | head -8
