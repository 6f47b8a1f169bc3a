# One-exchange-per-reflector tridiagonalisation: eig parity tests, eig timing by G,
# then the double-buffered factor state (overlap/distributed parity, bench A/B).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_eig_variance.py -x -q --timeout 120 --timeout-method thread > gpurun_out/eig_tests.log 2>&1 || { tail -30 gpurun_out/eig_tests.log; exit 1; }
tail -1 gpurun_out/eig_tests.log
for g in 0 64 128 256; do
  KFAC_EIG_G=$g timeout -k 10 120 python tools/bench_eig.py 129 785 2048 > gpurun_out/eig_g$g.log 2>&1 || { cat gpurun_out/eig_g$g.log; exit 1; }
  echo "G=$g"; cat gpurun_out/eig_g$g.log
done
timeout -k 10 200 python tools/bench_eig.py 4097 > gpurun_out/eig_4097.log 2>&1 || { cat gpurun_out/eig_4097.log; exit 1; }
cat gpurun_out/eig_4097.log
bash tools/gpu/dbuf_ab.sh
