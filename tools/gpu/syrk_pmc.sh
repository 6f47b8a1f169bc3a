# PMC counters of the 64-tile SYRK launch (8-batch MLP job set) and its no-DMA ablation.
set -o pipefail
mkdir -p gpurun_out/spmc
export TMPDIR=/tmp
cd tools/microbench
for V in 0 1 3; do
  ./syrk_ab 8 $V > ../../gpurun_out/spmc/time_$V.log 2>&1 || exit 1
  cat ../../gpurun_out/spmc/time_$V.log
  i=0
  for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
           "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM GRBM_GUI_ACTIVE"; do
    i=$((i+1))
    timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d ../../gpurun_out/spmc/v${V}_p$i -o run -- ./syrk_ab 8 $V > /dev/null 2>&1
    rc=$?; [ $rc -le 2 ] || exit $rc
  done
done
cd ../..
python - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/spmc/v*_p*/**/run_counter_collection.csv", recursive=True)):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if "factor_tiles" in r["Kernel_Name"]:
            vals[r["Counter_Name"]].append(float(r["Counter_Value"]))
    print(f.split("/")[2], {k: "%.4g" % (sum(v) / len(v)) for k, v in vals.items()})
PY
