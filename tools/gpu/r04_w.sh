# Round 4: premise check -- a full tile with 3 of its 4 fragments loaded and split per stage
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04w
mkdir -p $O
for v in def ab4 def ab4; do
  L=bnn_kfac_amd/libkfac_hip.so; [ $v != def ] && L=ab_libs/$v/libkfac_hip.so
  BNN_KFAC_AMD_LIB=$L timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_$v.log 2>&1 || { tail -20 $O/alone_$v.log; exit 1; }
  echo "$v: $(python -c "import json;d=json.loads(open('$O/alone_$v.log').read().strip().splitlines()[-1]);print(round(d['x3_us_per_launch'],1), round(d['pass_ms'],4))")"
done
