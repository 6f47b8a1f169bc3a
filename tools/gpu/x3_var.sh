# x3 direct-load variants on the MLP group (tools/x3_probe.py at 16384 / 32768 rows):
# hazard-ordered asm split (default) vs compiler split (a0) vs 3-statement asm (a2),
# 3 waves/SIMD registers (o3) at 4 / 6 planned workgroups per CU; then PMC of default
set -o pipefail
mkdir -p gpurun_out/x3v
KFAC_TILES_X3=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/x3v/tests.log 2>&1 || { tail -40 gpurun_out/x3v/tests.log; exit 1; }
tail -1 gpurun_out/x3v/tests.log
for R in 16384 32768; do
  for L in kfac_hip kfac_hip_a0 kfac_hip_a2 kfac_hip_o3; do
    BNN_KFAC_AMD_LIB=$PWD/bnn_kfac_amd/lib$L.so timeout -k 10 120 python tools/x3_probe.py $R > gpurun_out/x3v/p_${L}_$R.log 2>&1 || { tail -20 gpurun_out/x3v/p_${L}_$R.log; exit 1; }
    grep "x3:" gpurun_out/x3v/p_${L}_$R.log
  done
  for W in 5 6; do
    KFAC_X3_WGS=$W BNN_KFAC_AMD_LIB=$PWD/bnn_kfac_amd/libkfac_hip_o3.so timeout -k 10 120 python tools/x3_probe.py $R > gpurun_out/x3v/p_o3w${W}_$R.log 2>&1 || exit 1
    echo "wgs=$W $(grep 'x3:' gpurun_out/x3v/p_o3w${W}_$R.log)"
  done
done
export TMPDIR=/tmp
OUT=gpurun_out/x3v/pmc
mkdir -p $OUT
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS"; do
  name=$(echo $C | cut -d' ' -f1)
  timeout -k 10 -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "kfac_factor_tiles_x3" --output-format csv \
      -d $OUT/pmc_$name -o run -- python3 tools/x3_probe.py 32768 > $OUT/pmc_$name.log 2>&1
  rc=$?; echo "pmc $name rc=$rc"; [ $rc -le 2 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob("gpurun_out/x3v/pmc/pmc_*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        tot[row["Counter_Name"]] += float(row["Counter_Value"]); n[row["Counter_Name"]] += 1
for k in sorted(tot): print(k, tot[k], n[k])
wc = tot["SQ_WAVE_CYCLES"]
print("parked", tot["SQ_WAIT_ANY"]/wc, "issue-stall", tot["SQ_WAIT_INST_ANY"]/wc, "active", tot["SQ_ACTIVE_INST_ANY"]/wc,
      "mfma busy", tot["SQ_VALU_MFMA_BUSY_CYCLES"]/1024/(tot["GRBM_GUI_ACTIVE"]/8))
PY
