# Round 4: whole K-ranges per XCD with the thin-row pairs (interleave x splits 8 / 16 / default)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04z
mkdir -p $O
for cfg in "0 0" "1 8" "1 0" "1 16" "0 0" "1 8"; do
  set -- $cfg
  SP=""; [ $2 != 0 ] && SP=$2
  KFAC_X3_INTERLEAVE=$1 KFAC_SYRK_SPLITS=$SP timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_i$1_s$2.log 2>&1 || { tail -20 $O/alone_i$1_s$2.log; exit 1; }
  echo "i$1 s$2: $(python -c "import json;d=json.loads(open('$O/alone_i$1_s$2.log').read().strip().splitlines()[-1]);print(round(d['x3_us_per_launch'],1), round(d['pass_ms'],4))")"
done
for cfg in "1 8" "0 0"; do
  set -- $cfg
  SP=""; [ $2 != 0 ] && SP=$2
  KFAC_X3_INTERLEAVE=$1 KFAC_SYRK_SPLITS=$SP timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-include-regex "kfac_factor_tiles_x3" --output-format csv -d $O/pmc_i$1_s$2 -o run -- python tools/syrk_alone.py mlp 5 > $O/pmc_i$1_s$2.log 2>&1 || { echo "pmc rc=$?"; tail -5 $O/pmc_i$1_s$2.log; exit 1; }
done
python - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r04z/pmc_*/run_counter_collection.csv")):
    s = collections.defaultdict(float); d = collections.defaultdict(set)
    for r in csv.DictReader(open(f)):
        s[r["Counter_Name"]] += float(r["Counter_Value"]); d[r["Counter_Name"]].add(r["Dispatch_Id"])
    print(f.split("/")[2], {k: round(v / len(d[k])) for k, v in s.items()})
PY
