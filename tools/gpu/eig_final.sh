# Eigensolver round-2 check: parity tests, timings (values, vectors), rocprofv3 kernel
# stats at 785 and 4097 (csv), step-phase stamps at 785.
set -o pipefail
mkdir -p gpurun_out/eig_r02
timeout -k 10 300 python -u -m pytest tests/test_gpu_eig_variance.py tests/test_gpu_wide.py -x -q --timeout 120 --timeout-method thread > gpurun_out/eig_r02/tests.log 2>&1 || { tail -30 gpurun_out/eig_r02/tests.log; exit 1; }
tail -1 gpurun_out/eig_r02/tests.log
timeout -k 10 200 python tools/bench_eig.py 129 785 2048 4097 > gpurun_out/eig_r02/values.log 2>&1 || { cat gpurun_out/eig_r02/values.log; exit 1; }
EIG_VECS=1 timeout -k 10 200 python tools/bench_eig.py 785 2048 > gpurun_out/eig_r02/vectors.log 2>&1 || { cat gpurun_out/eig_r02/vectors.log; exit 1; }
KFAC_EIG_PROF=1 timeout -k 10 100 python tools/bench_eig.py 785 > gpurun_out/eig_r02/phases.log 2>&1 || { cat gpurun_out/eig_r02/phases.log; exit 1; }
grep -hv amdgpu gpurun_out/eig_r02/values.log gpurun_out/eig_r02/vectors.log
grep "us/step" gpurun_out/eig_r02/phases.log | tail -1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/eig_r02/prof -o eig -- python3 $GRAFT_REPO_ROOT/tools/bench_eig.py 785 4097 > $GRAFT_REPO_ROOT/gpurun_out/eig_r02/prof.log 2>&1 || echo "rocprofv3 exit $? (see prof.log)"
ls $GRAFT_REPO_ROOT/gpurun_out/eig_r02/prof
