# PMC counters of one LeNet conv SYRK job (conv_ab job index $1, default 2 = conv2 A).
set -o pipefail
mkdir -p gpurun_out/cpmc
export TMPDIR=/tmp
J=${1:-2}
cd tools/microbench
./conv_ab $J || exit 1
i=0
for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
         "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_SALU" \
         "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM"; do
  i=$((i+1))
  timeout -s KILL 60 rocprofv3 --pmc $C --output-format csv -d ../../gpurun_out/cpmc/p$i -o run -- ./conv_ab $J > /dev/null 2>&1
  rc=$?; [ $rc -le 2 ] || exit $rc
done
cd ../..
python - <<'PY'
import csv, glob, collections
acc = collections.defaultdict(list)
for f in sorted(glob.glob("gpurun_out/cpmc/p*/**/run_counter_collection.csv", recursive=True)):
    for r in csv.DictReader(open(f)):
        if "conv" in r["Kernel_Name"]:
            acc[r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(acc.items()):
    print(f"{k:28s} {sum(v)/len(v):14.0f}  ({len(v)} dispatches)")
PY
