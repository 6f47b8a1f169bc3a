#!/bin/bash
# Profile recipe (run on the GPU box from the repo root):
#   kernel trace + stats of the bench, then separate --pmc passes (gfx950 rules:
#   FETCH_SIZE and WRITE_SIZE in separate passes, no --pmc with tracing domains).
# Output under gpurun_out/prof_<tag>/ ; summaries are copied into profiles/ by hand.
set -u
TAG=${1:-r01}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
BENCH=${BENCH:-"python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-serial --no-other-configs"}  # (the pipelined loop only: its launches are the roofline line's) override for other configs
ok() { [ "$1" -le 2 ]; }   # 0 ok, 1/2 = profiler/usage error (no GPU fault)

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BENCH > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; ok $rc || exit $rc
timeout -k 10 120 rocprofv3 -L > $OUT/counters.txt 2>&1
for C in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM" "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo $C | tr ' ' '_')
  timeout -k 10 300 rocprofv3 --pmc $C --kernel-include-regex "kfac_factor|inv_|kfac_quad" --output-format csv \
      -d $OUT/pmc_$name -o run -- $BENCH > $OUT/pmc_$name.log 2>&1
  rc=$?; echo "pmc $name rc=$rc"; ok $rc || exit $rc
done
