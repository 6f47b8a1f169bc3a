# Round 4: split residuals as v_pk_add_f32 (A/B: parity + SYRK alone + bench)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ab
mkdir -p $O
A=ab_libs/pk/libkfac_hip.so
BNN_KFAC_AMD_LIB=$A timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_boundary.py tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread > $O/pk_tests.log 2>&1 || { tail -30 $O/pk_tests.log; exit 1; }
echo "pk parity: $(tail -1 $O/pk_tests.log)"
for v in def pk def pk; do
  L=bnn_kfac_amd/libkfac_hip.so; [ $v != def ] && L=$A
  BNN_KFAC_AMD_LIB=$L timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_$v.log 2>&1 || { tail -20 $O/alone_$v.log; exit 1; }
  echo "$v: $(python -c "import json;d=json.loads(open('$O/alone_$v.log').read().strip().splitlines()[-1]);print(round(d['x3_us_per_launch'],1), round(d['pass_ms'],4))")"
done
for v in def pk def pk; do
  L=bnn_kfac_amd/libkfac_hip.so; [ $v != def ] && L=$A
  BNN_KFAC_AMD_LIB=$L timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-serial > $O/bench_$v.log 2>&1 || { tail -20 $O/bench_$v.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_$v.log').read().strip().splitlines()[-1]);print('bench $v', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_us'],1))"
done
