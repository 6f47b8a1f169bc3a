# counters of the conv bf16x3 kernels on the LeNet-5 bench loop (separate --pmc passes)
# (KRE: kernel regex, default conv_x3; BNN_KFAC_AMD_LIB picks a library variant)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:?set TAG}
mkdir -p $O
KRE=${KRE:-conv_x3}
B="python3 bench.py --config lenet --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-serial --no-eig --no-other-configs"
i=0
for C in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_SMEM" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_BRANCH GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "$KRE" --output-format csv -d $O/pmc$i -o run -- $B > $O/pmc$i.log 2>&1 || { tail -20 $O/pmc$i.log; exit 1; }
done
python3 - <<PY
import csv, glob, collections
for f in sorted(glob.glob("$O/pmc*/run_counter_collection.csv")):
    v = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        v[(r["Kernel_Name"].split("(")[0][-24:], r["Counter_Name"])].append(float(r["Counter_Value"]))
    for k, x in sorted(v.items()):
        print(f"{k[0]:24s} {k[1]:32s} mean {sum(x)/len(x):.4g}  n {len(x)}")
PY
