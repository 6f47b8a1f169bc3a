# kernel trace of a short bench run (for inter-kernel gap analysis: tools/gaps.py)
set -o pipefail
mkdir -p gpurun_out/trace_gaps
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_gaps -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/trace_gaps/log 2>&1 || exit $?
find gpurun_out/trace_gaps -name "*.csv" | head
