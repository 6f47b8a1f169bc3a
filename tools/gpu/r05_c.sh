# Round 5: CU-tile microbench variant matrix (VALU pattern, lazy B reads, spread loads)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05c
mkdir -p $O
timeout -k 10 120 ./tools/microbench/cut_mb > $O/cut_mb.log 2>&1; echo "cut_mb rc $?"; cat $O/cut_mb.log
