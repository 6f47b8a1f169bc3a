# Round 5: the data-parallel pass's collective on the inversion's side stream --
# distributed GPU tests (gloo world 2 on one device, RCCL world 1), the 2-rank
# shared-device bench, and the 1-GPU line unchanged
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bo
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_distributed.py > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
grep -E "passed|failed|skipped" $O/tests.log | tail -3
timeout -k 10 300 python3 bench.py --gpus 2 --shared-device --steps 10 --warmup 3 --no-serial --images 32768 > $O/bench_shared.log 2>&1 || { tail -20 $O/bench_shared.log; exit 1; }
tail -1 $O/bench_shared.log | cut -c1-600
