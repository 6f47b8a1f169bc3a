# PMC counters of kfac_factor_tiles_x3 on the MLP bench (one pass per counter group)
set -u
OUT=gpurun_out/x3pmc
mkdir -p $OUT
export TMPDIR=/tmp
# (kfac_factor_tiles_x3 is the default for the MNIST MLP factors)
BENCH="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-serial"
for C in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_WAVES GRBM_GUI_ACTIVE"; do
  name=$(echo $C | cut -d' ' -f1)
  timeout -k 10 -s KILL 240 rocprofv3 --pmc $C --kernel-include-regex "kfac_factor_tiles_x3" --output-format csv \
      -d $OUT/pmc_$name -o run -- $BENCH > $OUT/pmc_$name.log 2>&1
  rc=$?; echo "pmc $name rc=$rc"; [ $rc -le 2 ] || exit $rc
done
python3 - <<'PY'
import csv, glob, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob("gpurun_out/x3pmc/pmc_*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        tot[row["Counter_Name"]] += float(row["Counter_Value"]); n[row["Counter_Name"]] += 1
for k in sorted(tot): print(k, tot[k], n[k])
PY
