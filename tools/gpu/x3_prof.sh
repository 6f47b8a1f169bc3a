# FETCH_SIZE calibration of the x3 kernel's access pattern, then the MLP profile
# (trace + PMC passes) of the default build -> profiles/r03 via summarize.py
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
for C in FETCH_SIZE; do
  KFAC_TILES_X3=1 timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "kfac_factor_tiles_x3" --output-format csv \
      -d gpurun_out/calib/pmc -o run -- python3 tools/fetch_calib.py > gpurun_out/calib/calib.log 2>&1
  rc=$?; echo "calib rc=$rc"; [ $rc -le 2 ] || exit $rc
done
python3 - <<'PY'
import csv, glob
v = [float(r["Counter_Value"]) for f in glob.glob("gpurun_out/calib/pmc/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(f))]
print("FETCH_SIZE KiB per launch:", v)
ob = [l for l in open("gpurun_out/calib/calib.log") if l.startswith("operand bytes")]
print(ob)
PY
bash profiles/collect.sh r03 > gpurun_out/prof_r03.log 2>&1 || { tail -20 gpurun_out/prof_r03.log; exit 1; }
tail -8 gpurun_out/prof_r03.log
