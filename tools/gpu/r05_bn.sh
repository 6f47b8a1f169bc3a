# Round 5: the step against its parts on the final kernels (pairs, prio 0, ordering events)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bn
mkdir -p $O
timeout -k 10 300 python3 tools/probe_step_parts.py 200 3 > $O/parts.log 2>&1 || { tail -20 $O/parts.log; exit 1; }
tail -1 $O/parts.log
