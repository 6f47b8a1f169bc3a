# Round 4: the factor pass alone (no inversion beside) under the timing A/B builds
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04e
mkdir -p $O
for v in default noload nosplit mfmaonly; do
  if [ $v = default ]; then L=bnn_kfac_amd/libkfac_hip.so; else L=ab_libs/$v/libkfac_hip.so; fi
  echo -n "$v: "; BNN_KFAC_AMD_LIB=$L timeout -k 10 120 python tools/syrk_alone.py mlp 20 2>&1 | tail -1
done
