set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_eig_variance.py tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/eig_tests.log 2>&1 || { tail -30 gpurun_out/eig_tests.log; exit 1; }
tail -1 gpurun_out/eig_tests.log
for g in 64 96 128 160 256; do
KFAC_EIG_PROF=1 KFAC_EIG_G=$g timeout -k 10 120 python tools/bench_eig.py 785 > gpurun_out/eigclk.log 2>&1 || { tail -5 gpurun_out/eigclk.log; exit 1; }
echo "G=$g $(grep 'us/step' gpurun_out/eigclk.log | tail -1)"
done
