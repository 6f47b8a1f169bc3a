# Round-3 re-entry check on HEAD: whole GPU suite, smoke, MLP / LeNet-5 / wide lines
set -o pipefail
mkdir -p gpurun_out/h0
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/h0/tests.log 2>&1 || { tail -40 gpurun_out/h0/tests.log; exit 1; }
tail -1 gpurun_out/h0/tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/h0/smoke.log 2>&1 || { tail -20 gpurun_out/h0/smoke.log; exit 1; }
tail -1 gpurun_out/h0/smoke.log
timeout -k 10 400 python bench.py > gpurun_out/h0/bench_mlp.log 2>&1 || exit 1
tail -1 gpurun_out/h0/bench_mlp.log | cut -c1-400
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline > gpurun_out/h0/bench_lenet.log 2>&1 || exit 1
tail -1 gpurun_out/h0/bench_lenet.log | cut -c1-300
timeout -k 10 300 python bench.py --config wide --no-cpu-baseline > gpurun_out/h0/bench_wide.log 2>&1 || exit 1
tail -1 gpurun_out/h0/bench_wide.log | cut -c1-300
