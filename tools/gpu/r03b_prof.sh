# FETCH_SIZE calibration of kfac_factor_tiles_x3's access pattern, then the MLP
# profile of the default build (trace + PMC passes) -> profiles/r03b via summarize.py
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/calib
KFAC_TILES_X3=1 timeout -k 10 -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "kfac_factor_tiles_x3" --output-format csv \
    -d gpurun_out/calib/pmc -o run -- python3 tools/fetch_calib.py > gpurun_out/calib/calib.log 2>&1
rc=$?; echo "calib rc=$rc"; [ $rc -le 2 ] || exit $rc
python3 - <<'PY' | tee gpurun_out/calib/fetch_calib.txt
import csv, glob
v = [float(r["Counter_Value"]) for f in glob.glob("gpurun_out/calib/pmc/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(f))]
ob = [int(l.split()[-1]) for l in open("gpurun_out/calib/calib.log") if l.startswith("operand bytes")]
print("FETCH_SIZE KiB per launch:", v)
print("operand bytes:", ob)
if v and ob:
    print("scale (bytes per FETCH_SIZE byte):", ob[0] / (sum(v) / len(v) * 1024))
PY
[ "${CALIB_ONLY:-0}" = 1 ] && exit 0
bash profiles/collect.sh r03b > gpurun_out/prof_r03b.log 2>&1 || { tail -20 gpurun_out/prof_r03b.log; exit 1; }
tail -8 gpurun_out/prof_r03b.log
