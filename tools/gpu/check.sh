# GPU end check (gpurun -- 'TAG=r06x bash tools/gpu/check.sh'):
#   the whole GPU suite, smoke(), the bench as the driver runs it (--steps 20 --warmup 5),
#   then (PROF=1) the rocprofv3 kernel trace + PMC passes of each config's bench loop and
#   the eigensolver's kernel trace.  Logs under gpurun_out/$TAG/.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:?set TAG}
mkdir -p $O
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
  tail -2 $O/gpu_tests.log
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
  tail -1 $O/smoke.log
fi
if [ "${BENCH:-1}" = 1 ]; then
  timeout -k 10 500 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_mlp.log 2>&1 || { tail -20 $O/bench_mlp.log; exit 1; }
  python tools/line_summary.py $O/bench_mlp.log
fi
if [ "${PROF:-0}" = 1 ]; then
  for c in ${PROF_CONFIGS:-mlp lenet wide}; do
    bash profiles/collect.sh ${TAG}_$c $c || exit 1
  done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/eig_trace -o run -- \
      python3 tools/bench_eig.py 785 4097 > $O/eig_trace.log 2>&1 || { tail -20 $O/eig_trace.log; exit 1; }
fi
