# Round 4: x3 thin-row pairs (diagonal + edge tile per task): parity, SYRK alone, bench, timeline
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py tests/test_gpu_boundary.py -x -q --timeout 200 --timeout-method thread > $O/pair_tests.log 2>&1 || { tail -30 $O/pair_tests.log; exit 1; }
echo "parity: $(tail -1 $O/pair_tests.log)"
for i in 1 2; do
  timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_$i.log 2>&1 || { tail -20 $O/alone_$i.log; exit 1; }
  echo "alone: $(tail -1 $O/alone_$i.log)"
done
for i in 1 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-serial > $O/bench_$i.log 2>&1 || { tail -20 $O/bench_$i.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$i.log').read().strip().splitlines()[-1]);print('bench', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_us'],1), round(d['roofline']['frac'],3), d['breakdown']['host_issue_ms_per_step'])"
done
BNN_KFAC_AMD_LIB=ab_libs/stamps/libkfac_hip.so timeout -k 10 200 python tools/x3_stamps.py mlp > $O/stamps.json 2>&1 || { tail -20 $O/stamps.json; exit 1; }
grep -v amdgpu $O/stamps.json | python -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({k: d[k] for k in d if k.startswith('mask') or k in ('launch_span_us','end_us_p0_p10_p50_p90_p100','blocks')}))"
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "kfac_factor_tiles_x3" --output-format csv -d $O/pmc -o run -- python tools/syrk_alone.py mlp 5 > $O/pmc.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc.log; exit 1; }
python - <<'PY'
import csv, collections
s = collections.defaultdict(float); d = collections.defaultdict(set)
for r in csv.DictReader(open("gpurun_out/r04r/pmc/run_counter_collection.csv")):
    s[r["Counter_Name"]] += float(r["Counter_Value"]); d[r["Counter_Name"]].add(r["Dispatch_Id"])
print({k: round(v / len(d[k])) for k, v in s.items()})
PY
