# Round-4 end check (second) on the committed tree: GPU suite, smoke, the default bench line (as
# the driver runs it), LeNet-5 and wide lines, kernel trace of the default MLP bench
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/r04_end2
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r04_end2/gpu_tests.log 2>&1 || { tail -40 gpurun_out/r04_end2/gpu_tests.log; exit 1; }
tail -1 gpurun_out/r04_end2/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r04_end2/smoke.log 2>&1 || { tail -20 gpurun_out/r04_end2/smoke.log; exit 1; }
tail -1 gpurun_out/r04_end2/smoke.log
timeout -k 10 500 python bench.py > gpurun_out/r04_end2/bench_mlp.log 2>&1 || exit 1
tail -1 gpurun_out/r04_end2/bench_mlp.log | cut -c1-300
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline > gpurun_out/r04_end2/bench_lenet.log 2>&1 || exit 1
tail -1 gpurun_out/r04_end2/bench_lenet.log | cut -c1-200
timeout -k 10 300 python bench.py --config wide --no-cpu-baseline > gpurun_out/r04_end2/bench_wide.log 2>&1 || exit 1
tail -1 gpurun_out/r04_end2/bench_wide.log | cut -c1-200
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r04_end2/trace_mlp -o run -- python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e > gpurun_out/r04_end2/trace_mlp.log 2>&1 || exit 1
head -6 gpurun_out/r04_end2/trace_mlp/run_kernel_stats.csv | cut -c1-150
