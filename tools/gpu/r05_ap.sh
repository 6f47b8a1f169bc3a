# Round 5: 2 vs 3 side-reduce accumulator buffers on the MLP loop (tools/probe_acc_bufs.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ap
mkdir -p $O
timeout -k 10 300 python3 tools/probe_acc_bufs.py 200 3 > $O/acc_bufs.log 2>&1 || { tail -20 $O/acc_bufs.log; exit 1; }
cat $O/acc_bufs.log
