# Round 5: the pipelined MLP step against its parts (tools/probe_step_parts.py)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ak
mkdir -p $O
timeout -k 10 300 python3 tools/probe_step_parts.py 200 3 > $O/parts.log 2>&1 || { tail -20 $O/parts.log; exit 1; }
cat $O/parts.log
