# Round 4: narrow x3 jobs' extra K-splits (KFAC_X3_NARROW 4 vs 1) on the MLP line, and
# per-kernel times of the wide inversion with / without the register-prefetched bulk updates
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ah
mkdir -p $O
for nf in 4 1 4 1; do
  KFAC_X3_NARROW=$nf timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-e2e --no-serial > $O/bench_n$nf.log 2>&1 || { tail -20 $O/bench_n$nf.log; exit 1; }
  echo "narrow x$nf: $(python -c "import json;d=json.loads(open('$O/bench_n$nf.log').read().strip().splitlines()[-1]);print(round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['roofline']['achieved'],1))")"
done
for lib in new inv0; do
  L=bnn_kfac_amd/libkfac_hip.so; [ $lib = inv0 ] && L=ab_libs/inv0/libkfac_hip.so
  BNN_KFAC_AMD_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$lib -o run -- python tools/step_split.py 4 wide > $O/prof_$lib.log 2>&1 || { tail -20 $O/prof_$lib.log; exit 1; }
  f=$(find $O/prof_$lib -name "*kernel_stats.csv" | head -1)
  echo "== $lib"; python -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows:
    if 'inv_' in r['Name'] or 'xtx' in r['Name']:
        print(r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), round(float(r['TotalDurationNs'])/1e6,2))
"
done
