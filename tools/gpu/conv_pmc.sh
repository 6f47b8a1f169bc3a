# counters of kfac_factor_conv_x3 on the LeNet-5 bench loop (separate --pmc passes)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:?set TAG}
mkdir -p $O
B="python3 bench.py --config lenet --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-serial --no-eig"
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_SALU SQ_INSTS_VMEM" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "conv_x3" --output-format csv -d $O/pmc$i -o run -- $B > $O/pmc$i.log 2>&1 || { tail -20 $O/pmc$i.log; exit 1; }
done
python3 - <<PY
import csv, glob, collections
for f in sorted(glob.glob("$O/pmc*/run_counter_collection.csv")):
    v = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        v[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, x in sorted(v.items()):
        print(f"{k:32s} mean {sum(x)/len(x):.4g}  n {len(x)}")
PY
