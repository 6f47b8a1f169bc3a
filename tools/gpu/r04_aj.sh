# Round 4: inversion wave / stream priority 0 vs the defaults, MLP and LeNet-5 lines
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04aj
mkdir -p $O
for cfg in lenet mlp; do
  for v in "-1 3" "0 0" "-1 3" "0 0" "-1 0"; do
    set -- $v
    t=${cfg}_s$1_w$2
    KFAC_INV_STREAM_PRIO=$1 KFAC_INV_PRIO=$2 timeout -k 10 200 python bench.py --config $cfg --steps 100 --warmup 10 --no-cpu-baseline --no-e2e --no-serial > $O/bench_$t.log 2>&1 || { tail -20 $O/bench_$t.log; exit 1; }
    echo "$t: $(python -c "import json;d=json.loads(open('$O/bench_$t.log').read().strip().splitlines()[-1]);b=d['breakdown'];print(round(d['value']/1e6,3), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_us'],1), round(b['invert_ms_per_step'],3))")"
  done
done
