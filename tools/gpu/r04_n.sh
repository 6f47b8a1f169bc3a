# Round 4: L2 warm-up prefetch in the x3 loop (A/B: parity, SYRK alone, bench)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
A=ab_libs/pf/libkfac_hip.so
BNN_KFAC_AMD_LIB=$A timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py -x -q --timeout 200 --timeout-method thread > $O/pf_tests.log 2>&1 || { tail -30 $O/pf_tests.log; exit 1; }
echo "pf parity: $(tail -1 $O/pf_tests.log)"
for v in def pf def pf; do
  L=bnn_kfac_amd/libkfac_hip.so; [ $v = pf ] && L=$A
  BNN_KFAC_AMD_LIB=$L timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_$v.log 2>&1 || { tail -20 $O/alone_$v.log; exit 1; }
  echo "alone $v: $(tail -1 $O/alone_$v.log)"
done
BNN_KFAC_AMD_LIB=$A timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-serial > $O/bench_pf.log 2>&1 || { tail -20 $O/bench_pf.log; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_pf.log').read().strip().splitlines()[-1]);print('bench pf', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_us'],1), d['breakdown']['host_issue_ms_per_step'])"
