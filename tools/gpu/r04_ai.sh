# Round 4: inversion side-stream priority / wave priority / inversions in flight on the
# MLP line (the inversion now has a step of slack beside the next pass)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ai
mkdir -p $O
for v in "-1 3 2" "0 3 2" "-1 0 2" "0 0 2" "-1 0 3" "0 0 3" "-1 3 2" "0 0 2"; do
  set -- $v
  t=s$1_w$2_p$3
  KFAC_INV_STREAM_PRIO=$1 KFAC_INV_PRIO=$2 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --max-pending $3 --no-cpu-baseline --no-e2e --no-serial > $O/bench_$t.log 2>&1 || { tail -20 $O/bench_$t.log; exit 1; }
  echo "$t: $(python -c "import json;d=json.loads(open('$O/bench_$t.log').read().strip().splitlines()[-1]);b=d['breakdown'];print(round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_us'],1), round(b['invert_ms_per_step'],3))")"
done
