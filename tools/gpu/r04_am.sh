# Round 4: extra, shorter K-splits for the x3 thin-row pair units (KFAC_X3_PAIR_XS):
# parity, then the MLP line A/B and the per-workgroup end times
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04am
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py tests/test_gpu_boundary.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "parity: $(tail -1 $O/tests.log)"
for xs in 1 0; do
  KFAC_X3_PAIR_XS=$xs BNN_KFAC_AMD_LIB=ab_libs/stamps/libkfac_hip.so timeout -k 10 200 python tools/x3_stamps.py mlp > $O/stamps_xs$xs.json 2>&1 || { tail -20 $O/stamps_xs$xs.json; exit 1; }
  echo "== xs $xs"; grep -v amdgpu $O/stamps_xs$xs.json | python -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({k: d[k] for k in d if k not in ('workgroups_per_cu',)}))"
done
for xs in 1 0 1 0; do
  KFAC_X3_PAIR_XS=$xs timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-e2e --no-serial > $O/bench_xs$xs.log 2>&1 || { tail -20 $O/bench_xs$xs.log; exit 1; }
  echo "xs $xs: $(python -c "import json;d=json.loads(open('$O/bench_xs$xs.log').read().strip().splitlines()[-1]);print(round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_us'],1))")"
done
