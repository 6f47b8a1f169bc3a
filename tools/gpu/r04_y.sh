# Round 4: stream waits on host-settled events skipped (A/B), MLP bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04y
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_invert.py tests/test_gpu_invert_graph.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "tests: $(tail -1 $O/tests.log)"
for v in 1 0 1 0 1 0; do
  KFAC_SKIP_DONE_WAITS=$v timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-serial > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]);print('skip=$v', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_us'],1), d['breakdown']['host_issue_ms_per_step'])"
done
