# Round 4, first check: the new / tightened GPU tests, the full suite, smoke, the default
# bench line, then the exit-time SIGSEGV A/B under rocprofv3 --pmc:
# the same eig pass as profiles/r03_eig/fetch_size_4097.log (now with kfac_release at
# exit) and a control with no kfac library loaded at all.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_boundary.py tests/test_gpu_invert_graph.py \
  tests/test_gpu_eig_variance.py tests/test_gpu_distributed.py -x -v --timeout 200 --timeout-method thread \
  > $O/new_tests.log 2>&1 || { tail -60 $O/new_tests.log; exit 1; }
tail -2 $O/new_tests.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 500 python bench.py > $O/bench_mlp.log 2>&1 || { tail -20 $O/bench_mlp.log; exit 1; }
tail -1 $O/bench_mlp.log | cut -c1-400
export EIG_NO_CPU=1
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$O/eig_fetch -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_eig.py 4097 > $GRAFT_REPO_ROOT/$O/eig_fetch.log 2>&1; echo "eig under pmc: rc $?"
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$O/ctl_fetch -o run -- python3 $GRAFT_REPO_ROOT/tools/exit_control.py > $GRAFT_REPO_ROOT/$O/ctl_fetch.log 2>&1; echo "control under pmc: rc $?"
cd $GRAFT_REPO_ROOT
timeout -k 10 90 ./tools/microbench/x3w_mb > $O/x3w_mb.log 2>&1; echo "x3w_mb rc $?"; cat $O/x3w_mb.log
exit 0
