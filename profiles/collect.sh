#!/bin/bash
# Profile recipe (run on the GPU box from the repo root):
#   bash profiles/collect.sh <tag> <config>        config: mlp | lenet | wide
# kernel trace + stats of the config's single-GPU bench loop, then separate --pmc passes
# (gfx950 rules: FETCH_SIZE and WRITE_SIZE in separate passes, no --pmc with tracing
# domains, each pass its own run under a time limit).  Output under
# gpurun_out/prof_<tag>/; `python profiles/summarize.py <tag> <config>` (here, after the
# call) writes profiles/<tag>/ and profiles/pmc_<config>.json.
set -u
TAG=${1:?tag}
CFG=${2:-mlp}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# the pipelined loop only (its launches are the roofline line's); no eig leg (a
# cooperative launch + --pmc finalisation crash the profiler's exit)
BENCH="python3 bench.py --config $CFG --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-serial --no-other-configs --no-eig"
ok() { [ "$1" -eq 0 ]; }

timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- $BENCH > $OUT/trace.log 2>&1
rc=$?; echo "trace rc=$rc"; ok $rc || exit $rc
for C in FETCH_SIZE WRITE_SIZE "SQ_INSTS_VALU_MFMA_MOPS_F32 SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE" \
         "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY" "SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM" "TCC_HIT_sum TCC_MISS_sum"; do
  name=$(echo $C | tr ' ' '_')
  timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "kfac_factor|inv_" --output-format csv \
      -d $OUT/pmc_$name -o run -- $BENCH > $OUT/pmc_$name.log 2>&1
  rc=$?; echo "pmc $name rc=$rc"; ok $rc || exit $rc
done
