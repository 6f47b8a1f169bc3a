# Round 5: the select-free elimination (v_rcp_f64 + Newton, pivot by readlane, no SGPR
# spills) as committed: inversion / eig / golden / C2 / factor parity, the diagonal
# microbench, the inversion alone
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05v
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_invert.py tests/test_gpu_invert_graph.py tests/test_gpu_c2.py tests/test_gpu_golden_r02.py tests/test_gpu_eig_variance.py tests/test_gpu_wide.py tests/test_gpu_distributed.py tests/test_gpu_boundary.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 60 ./tools/microbench/diag_mb > $O/diag_mb.log 2>&1 || { tail -5 $O/diag_mb.log; exit 1; }
cat $O/diag_mb.log
timeout -k 10 200 python tools/probe_invert.py 300 tree > $O/invert.log 2>&1 || { tail -5 $O/invert.log; exit 1; }
cat $O/invert.log
