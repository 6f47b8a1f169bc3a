# Round 5: the queued wide-pass parity test, then the MLP bench's rocprofv3 kernel stats
# and PMC passes on the final tree (profiles/collect.sh, tag r05final)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ax
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/wide_tests.log 2>&1 || { tail -30 $O/wide_tests.log; exit 1; }
grep -E "passed|failed" $O/wide_tests.log | tail -6
bash profiles/collect.sh r05final || exit 1
