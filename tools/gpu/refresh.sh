# Round re-entry check: GPU parity suite, then the committed profile set and bench lines.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_tests.log 2>&1; rc=$?
tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
timeout -k 10 900 bash profiles/collect.sh r01 || exit $?
timeout -k 10 600 python bench.py > gpurun_out/bench_mlp.log 2>&1 || exit $?
tail -1 gpurun_out/bench_mlp.log | cut -c1-400
timeout -k 10 600 python bench.py --config lenet --steps 5 --warmup 2 > gpurun_out/bench_lenet.log 2>&1 || exit $?
timeout -k 10 600 python bench.py --config wide --steps 3 --warmup 1 --images 16384 > gpurun_out/bench_wide.log 2>&1 || exit $?
echo done
