# Round 4: wide MLP with the x3 SYRK (thin-row pairs) instead of the split pass
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04aa
mkdir -p $O
for v in 0 1 0; do
  KFAC_SYRK3=$v timeout -k 10 400 python bench.py --config wide --no-cpu-baseline --no-e2e --no-serial > $O/bench_wide_s3$v.log 2>&1 || { tail -20 $O/bench_wide_s3$v.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_wide_s3$v.log').read().strip().splitlines()[-1]);r=d['roofline'];print('syrk3=$v', round(d['value']/1e6,4), round(d['ms_per_step'],3), r['kernel'], round(r['avg_launch_us'],1), round(r['frac'],3), d['breakdown'])"
done
