# Round 4: practical MFMA ceiling (register-only microbench), the x3 pass's balance probe
# (every tile on the full-tile loop, with and without loads/split) and the split-pass
# route (KFAC_SYRK3=1) for the MNIST MLP
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 120 ./ab_libs/mfma_peak > $O/mfma_peak.log 2>&1 || { cat $O/mfma_peak.log; exit 1; }
cat $O/mfma_peak.log
for v in ab3 ab3full ab0full; do
  BNN_KFAC_AMD_LIB=ab_libs/$v/libkfac_hip.so timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_$v.log 2>&1 || { tail -20 $O/alone_$v.log; exit 1; }
  echo "alone $v: $(tail -1 $O/alone_$v.log)"
done
timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_def.log 2>&1 || { tail -20 $O/alone_def.log; exit 1; }
echo "alone def: $(tail -1 $O/alone_def.log)"
KFAC_SYRK3=1 timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_syrk3.log 2>&1 || { tail -20 $O/alone_syrk3.log; exit 1; }
echo "alone syrk3: $(tail -1 $O/alone_syrk3.log)"
