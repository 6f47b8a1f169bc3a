# Round 5: the MLP inversion alone on 64-tiles (13 merged steps) vs 32-tiles (25)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bk
mkdir -p $O
for r in 1 2; do
timeout -k 10 120 python3 tools/probe_invert.py 300 t32 >> $O/invert.log 2>&1 || { tail -5 $O/invert.log; exit 1; }
KFAC_INV_TILE=64 timeout -k 10 120 python3 tools/probe_invert.py 300 t64 >> $O/invert.log 2>&1 || { tail -5 $O/invert.log; exit 1; }
done
grep median $O/invert.log
