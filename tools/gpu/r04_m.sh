# Round 4: x3 task order with whole K-ranges per XCD (KFAC_X3_INTERLEAVE) at several
# split counts; L2 hit/miss of the best against the default
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
BNN_KFAC_AMD_LIB=ab_libs/stamps/libkfac_hip.so KFAC_X3_INTERLEAVE=1 timeout -k 10 200 python tools/x3_stamps.py mlp > $O/stamps_inter.json 2>&1 || { tail -20 $O/stamps_inter.json; exit 1; }
for cfg in "0 0" "1 0" "1 8" "1 16" "0 16" "1 24"; do
  set -- $cfg
  n=i$1_s$2
  if [ $2 = 0 ]; then SP=""; else SP=$2; fi
  KFAC_X3_INTERLEAVE=$1 KFAC_SYRK_SPLITS=$SP timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_$n.log 2>&1 || { tail -20 $O/alone_$n.log; exit 1; }
  echo "$n: $(tail -1 $O/alone_$n.log)"
done
for v in "0" "1"; do
  KFAC_X3_INTERLEAVE=$v timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "kfac_factor_tiles_x3" --output-format csv -d $O/pmc_i$v -o run -- python tools/syrk_alone.py mlp 5 > $O/pmc_i$v.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc_i$v.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r04m/pmc_*/run_counter_collection.csv")):
    s = collections.defaultdict(float); d = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        s[r["Counter_Name"]] += float(r["Counter_Value"]); d[r["Counter_Name"]].add(r["Dispatch_Id"])
    print(f.split("/")[2], {k: round(v / len(d[k])) for k, v in s.items()})
PY
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-serial > $O/trace_bench.log 2>&1 || { echo "trace rc=$?"; tail -5 $O/trace_bench.log; exit 1; }
python tools/trace_gaps.py $(ls $O/trace/*kernel_trace.csv | head -1) 3.0 > $O/trace_gaps.txt 2>&1 || { cat $O/trace_gaps.txt; exit 1; }
cat $O/trace_gaps.txt
for lf in 4 8; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-serial --launch-first $lf > $O/bench_lf$lf.log 2>&1 || { tail -20 $O/bench_lf$lf.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_lf$lf.log').read().strip().splitlines()[-1]);print('lf$lf', round(d['value']/1e6,2), round(d['ms_per_step'],4), d['breakdown']['host_issue_ms_per_step'])"
done
