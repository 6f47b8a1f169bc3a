# Kernel timeline of the MLP bench (pipelined steps) under rocprofv3 --kernel-trace.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
LF=${LF:-16}
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/tl -o run -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline --no-e2e --no-serial --launch-first $LF > gpurun_out/tl.log 2>&1 || { tail -5 gpurun_out/tl.log; exit 1; }
f=$(find gpurun_out/tl -name "*kernel_trace.csv" | head -1)
python tools/timeline.py $f 140 > gpurun_out/timeline.txt
tail -1 gpurun_out/tl.log | cut -c1-200
head -3 $f | cut -c1-400
