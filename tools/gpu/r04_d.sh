# Round 4: what bounds kfac_factor_tiles_x3 in production (timing A/B builds, results
# wrong by construction): no reloads / no split / neither, on the default MLP bench line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
for v in default noload nosplit mfmaonly; do
  if [ $v = default ]; then L=bnn_kfac_amd/libkfac_hip.so; else L=ab_libs/$v/libkfac_hip.so; fi
  BNN_KFAC_AMD_LIB=$L timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-e2e --no-serial > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]);r=d['roofline'];print('$v', round(d['value']/1e6,2),'M img/s', round(d['ms_per_step'],4),'ms', r['kernel'], round(r['avg_launch_us'],1),'us', round(r['frac'],3))"
done
