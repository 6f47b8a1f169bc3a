# Round 5: phase stamps of the merged inversion steps' critical workgroup (MLP, alone)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05at
mkdir -p $O
BNN_KFAC_AMD_LIB=ab_libs/invstamps/libkfac_hip.so timeout -k 10 200 python3 tools/probe_inv_stamps.py 20 > $O/stamps.log 2>&1 || { tail -20 $O/stamps.log; exit 1; }
cat $O/stamps.log
