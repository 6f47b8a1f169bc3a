# kernel trace of a short LeNet-5 bench run (per-family SYRK durations)
set -o pipefail
mkdir -p gpurun_out/trace_lenet
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/trace_lenet -o run -- python3 bench.py --config lenet --steps 2 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/trace_lenet/log 2>&1 || exit $?
tail -1 gpurun_out/trace_lenet/log | cut -c1-300
