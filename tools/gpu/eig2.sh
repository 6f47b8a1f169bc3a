# Eigensolver: parity tests, timing by size, and rocprofv3 kernel stats at 785 / 4097.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_eig_variance.py tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/eig_tests.log 2>&1 || { tail -30 gpurun_out/eig_tests.log; exit 1; }
tail -1 gpurun_out/eig_tests.log
timeout -k 10 200 python tools/bench_eig.py 129 785 2048 4097 > gpurun_out/eig_t.log 2>&1 || { cat gpurun_out/eig_t.log; exit 1; }
grep -v amdgpu gpurun_out/eig_t.log
EIG_VECS=1 timeout -k 10 200 python tools/bench_eig.py 785 2048 > gpurun_out/eig_v.log 2>&1 || { cat gpurun_out/eig_v.log; exit 1; }
grep -v amdgpu gpurun_out/eig_v.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/eigprof -o eig -- python3 $GRAFT_REPO_ROOT/tools/bench_eig.py 785 4097 > $GRAFT_REPO_ROOT/gpurun_out/eigprof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/gpurun_out/eigprof.log; exit 1; }
find $GRAFT_REPO_ROOT/gpurun_out/eigprof -name "*kernel_stats.csv" | head -3 | xargs -I{} sh -c 'echo {}; head -12 {}'
