# Round 5: the pipelined MLP step against its parts again (inversion priority 0, ordering
# events): full / side reduce only / reduce on the caller's stream / launches only
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bc
mkdir -p $O
timeout -k 10 300 python3 tools/probe_step_parts.py 200 3 > $O/parts.log 2>&1 || { tail -20 $O/parts.log; exit 1; }
tail -1 $O/parts.log
