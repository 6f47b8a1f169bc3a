# Round 4: x3 timeline (pairs, one round, narrow jobs x4 splits) and the narrow-split A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ad
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "parity: $(tail -1 $O/tests.log)"
for nf in 4 1; do
  KFAC_X3_NARROW=$nf BNN_KFAC_AMD_LIB=ab_libs/stamps/libkfac_hip.so timeout -k 10 200 python tools/x3_stamps.py mlp > $O/stamps_n$nf.json 2>&1 || { tail -20 $O/stamps_n$nf.json; exit 1; }
  echo "== narrow x$nf"; grep -v amdgpu $O/stamps_n$nf.json | python -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({k: d[k] for k in d if k not in ('workgroups_per_cu',)}))"
done
for nf in 4 1 4 1; do
  KFAC_X3_NARROW=$nf timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_n$nf.log 2>&1 || { tail -20 $O/alone_n$nf.log; exit 1; }
  echo "narrow x$nf: $(python -c "import json;d=json.loads(open('$O/alone_n$nf.log').read().strip().splitlines()[-1]);print(round(d['x3_us_per_launch'],1), round(d['pass_ms'],4))")"
done
