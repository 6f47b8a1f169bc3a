# Round 5: the distributed GPU tests again (RCCL world 1 with the collective on the
# inversion's side stream)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05by
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "PASSED|FAILED|SKIPPED" $O/tests.log | cut -c1-120
