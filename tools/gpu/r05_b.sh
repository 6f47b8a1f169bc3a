# Round 5: interleaved CU-tile microbench variants; GPU suite on the cleaned factor.hip
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05b
mkdir -p $O
timeout -k 10 120 ./tools/microbench/cut_mb > $O/cut_mb.log 2>&1; echo "cut_mb rc $?"; cat $O/cut_mb.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
