# Round 4: host / GPU timeline of the pipelined MLP step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
timeout -k 10 200 python tools/step_timeline.py 40 > $O/timeline.log 2>&1 || { tail -20 $O/timeline.log; exit 1; }
tail -1 $O/timeline.log
timeout -k 10 200 python tools/step_timeline.py 40 > $O/timeline2.log 2>&1 || { tail -20 $O/timeline2.log; exit 1; }
tail -1 $O/timeline2.log
