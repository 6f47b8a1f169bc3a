# Round 4: per-workgroup timeline of the x3 launch (full build and MFMA-only build),
# and the planner at two dispatch rounds (KFAC_SYRK_ROUNDS=2)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04i
mkdir -p $O
for v in stamps stamps3; do
  BNN_KFAC_AMD_LIB=ab_libs/$v/libkfac_hip.so timeout -k 10 200 python tools/x3_stamps.py mlp > $O/$v.json 2>&1 || { tail -20 $O/$v.json; exit 1; }
  echo "== $v"; cat $O/$v.json
done
KFAC_SYRK_ROUNDS=2 timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_r2.log 2>&1 || { tail -20 $O/alone_r2.log; exit 1; }
echo "alone rounds2: $(tail -1 $O/alone_r2.log)"
