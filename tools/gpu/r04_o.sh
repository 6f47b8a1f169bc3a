# Round 4: queued inversions before invert() waits (KFAC.max_pending 2 / 3 / 4)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
for mp in 2 3 4 3 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-serial --max-pending $mp > $O/bench_mp$mp.log 2>&1 || { tail -20 $O/bench_mp$mp.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_mp$mp.log').read().strip().splitlines()[-1]);print('mp$mp', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_us'],1), d['breakdown']['host_issue_ms_per_step'], round(d['breakdown']['invert_ms_per_step'],3))"
done
