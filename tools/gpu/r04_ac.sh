# Round 4: wide SYRK (split pass + syrk3) task-order blocking vs fetch (is it fetch-bound?)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ac
mkdir -p $O
for cfg in "4 8" "8 8" "2 16" "16 16" "1 64" "4 8"; do
  set -- $cfg
  KFAC_S3_BI=$1 KFAC_S3_BJ=$2 timeout -k 10 300 python tools/syrk_alone.py wide 4 > $O/alone_$1_$2.log 2>&1 || { tail -20 $O/alone_$1_$2.log; exit 1; }
  echo "bi$1 bj$2: $(python -c "import json;d=json.loads(open('$O/alone_$1_$2.log').read().strip().splitlines()[-1]);print(round(d.get('syrk3_us_per_launch',0),1), round(d['pass_ms'],3))")"
done
for cfg in "4 8" "16 16" "1 64"; do
  set -- $cfg
  KFAC_S3_BI=$1 KFAC_S3_BJ=$2 timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "kfac_factor_syrk3" --output-format csv -d $O/pmc_$1_$2 -o run -- python tools/syrk_alone.py wide 2 > $O/pmc_$1_$2.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc_$1_$2.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r04ac/pmc_*/run_counter_collection.csv")):
    s = collections.defaultdict(float); d = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        s[r["Counter_Name"]] += float(r["Counter_Value"]); d[r["Counter_Name"]].add(r["Dispatch_Id"])
    print(f.split("/")[2], {k: round(v / len(d[k]) * 2 * 1024 / 1e9, 2) for k, v in s.items()}, "GB per launch (FETCH x2)")
PY
