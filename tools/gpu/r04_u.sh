# Round 4: x3 launch stagger (s_sleep per dispatch round) A/B
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
for st in 5 0 10 5 0 2; do
  KFAC_SYRK_STAGGER=$st timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_s$st.log 2>&1 || { tail -20 $O/alone_s$st.log; exit 1; }
  echo "stagger $st: $(python -c "import json;d=json.loads(open('$O/alone_s$st.log').read().strip().splitlines()[-1]);print(round(d['x3_us_per_launch'],1), round(d['pass_ms'],4))")"
done
for st in 5 0 5 0; do
  KFAC_SYRK_STAGGER=$st timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-serial > $O/bench_s$st.log 2>&1 || { tail -20 $O/bench_s$st.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_s$st.log').read().strip().splitlines()[-1]);print('bench stagger $st', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_us'],1))"
done
