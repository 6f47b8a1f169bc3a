# Round 4: pair units' extra K-splits, S = f + f / k (KFAC_X3_PAIR_XS = k), MLP line;
# then the new exactness test
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04an
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py -x -q --timeout 200 --timeout-method thread -k "extra_splits or thin_row or queued_pass or split_accumulator" > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "parity: $(tail -1 $O/tests.log)"
for k in 10 5 3 0 10 5 3 0; do
  KFAC_X3_PAIR_XS=$k timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-e2e --no-serial > $O/bench_k$k.log 2>&1 || { tail -20 $O/bench_k$k.log; exit 1; }
  echo "k $k: $(python -c "import json;d=json.loads(open('$O/bench_k$k.log').read().strip().splitlines()[-1]);print(round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_us'],1))")"
done
