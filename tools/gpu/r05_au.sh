# Round 5: the diagonal L block emitted by a non-critical task of the next step and Y's
# off-diagonal blocks cleared beside the first elimination -- GPU suite, then the MLP
# inversion alone (HEAD build vs this tree, alternating) and the phase stamps of both
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05au
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
for r in 1 2; do
BNN_KFAC_AMD_LIB=ab_libs/inv_head/libkfac_hip.so timeout -k 10 120 python3 tools/probe_invert.py 300 head >> $O/invert.log 2>&1 || { tail -5 $O/invert.log; exit 1; }
timeout -k 10 120 python3 tools/probe_invert.py 300 new >> $O/invert.log 2>&1 || { tail -5 $O/invert.log; exit 1; }
done
grep median $O/invert.log
BNN_KFAC_AMD_LIB=ab_libs/invstamps/libkfac_hip.so timeout -k 10 120 python3 tools/probe_inv_stamps.py 20 > $O/stamps_head.log 2>&1 || { tail -5 $O/stamps_head.log; exit 1; }
BNN_KFAC_AMD_LIB=ab_libs/invstamps2/libkfac_hip.so timeout -k 10 120 python3 tools/probe_inv_stamps.py 20 > $O/stamps_new.log 2>&1 || { tail -5 $O/stamps_new.log; exit 1; }
tail -1 $O/stamps_head.log
tail -1 $O/stamps_new.log
