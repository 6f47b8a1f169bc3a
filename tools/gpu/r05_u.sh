# Round 5: same-box A/B of the inversion alone: HEAD's elimination (orig), select-free
# + v_rcp_f64 (sf), and the in-tree build (sf, pivot by readlane, Y one column behind)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05u2
mkdir -p $O
for r in 1 2; do
for v in orig sf tree; do
if [ $v = tree ]; then unset BNN_KFAC_AMD_LIB; else export BNN_KFAC_AMD_LIB=$PWD/ab_libs/inv_$v/libkfac_hip.so; fi
timeout -k 10 200 python tools/probe_invert.py 300 $v >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
done
done
unset BNN_KFAC_AMD_LIB
grep median $O/ab.log
