# Round 5, first box: CU-tile microbench (split once per workgroup into LDS) beside the
# round-4 wave-tile microbench, then the GPU suite and the MLP bench line as a baseline.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05a
mkdir -p $O
timeout -k 10 120 ./tools/microbench/cut_mb > $O/cut_mb.log 2>&1; echo "cut_mb rc $?"; cat $O/cut_mb.log
timeout -k 10 120 ./tools/microbench/x3w_mb > $O/x3w_mb.log 2>&1; echo "x3w_mb rc $?"; cat $O/x3w_mb.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 300 python bench.py > $O/bench_mlp.log 2>&1 || { tail -20 $O/bench_mlp.log; exit 1; }
tail -1 $O/bench_mlp.log | cut -c1-600
