# Round 4: one x3 wave per SIMD (2 workgroups per CU planned) with and without loads
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
for cfg in "def 4" "def 2" "ab1 4" "ab1 2"; do
  set -- $cfg
  L=bnn_kfac_amd/libkfac_hip.so; [ $1 = ab1 ] && L=ab_libs/ab1/libkfac_hip.so
  BNN_KFAC_AMD_LIB=$L KFAC_SYRK_WGS=$2 timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_$1_w$2.log 2>&1 || { tail -20 $O/alone_$1_w$2.log; exit 1; }
  echo "$1 wgs$2: $(tail -1 $O/alone_$1_w$2.log)"
done
BNN_KFAC_AMD_LIB=ab_libs/stamps/libkfac_hip.so KFAC_SYRK_WGS=2 timeout -k 10 200 python tools/x3_stamps.py mlp > $O/stamps_w2.json 2>&1 || { tail -20 $O/stamps_w2.json; exit 1; }
grep -v amdgpu $O/stamps_w2.json | python -c "import json,sys; d=json.load(sys.stdin); print({k: d[k] for k in d if k.startswith('mask') or k in ('launch_span_us','clock_ghz_in_loop','workgroups_per_cu')})"
