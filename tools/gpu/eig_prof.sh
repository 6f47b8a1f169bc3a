# Step-phase breakdown of eig_tridiag (KFAC_EIG_PROF stamps) by size and grid, after
# the eig parity tests.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_eig_variance.py tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/eig_tests.log 2>&1 || { tail -30 gpurun_out/eig_tests.log; exit 1; }
tail -1 gpurun_out/eig_tests.log
for g in 0 64 128 256; do
  KFAC_EIG_PROF=1 KFAC_EIG_G=$g timeout -k 10 120 python tools/bench_eig.py 129 785 2048 > gpurun_out/eigp_$g.log 2>&1 || { tail -5 gpurun_out/eigp_$g.log; exit 1; }
  echo "G=$g"; grep -v amdgpu gpurun_out/eigp_$g.log | sort | uniq | sort -t' ' -k1,1 | awk '!seen[$1 $2 $3]++' | head -8
done
timeout -k 10 200 python tools/bench_eig.py 785 4097 > gpurun_out/eig_t.log 2>&1 || { cat gpurun_out/eig_t.log; exit 1; }
grep -v amdgpu gpurun_out/eig_t.log
