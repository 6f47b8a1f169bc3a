# Round 4: x3 thin-row pairs on / off x planner rounds (default / 1), SYRK alone + bench
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04s
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
echo "parity: $(tail -1 $O/tests.log)"
for cfg in "1 0" "0 0" "1 1" "0 1" "1 0" "0 0"; do
  set -- $cfg
  R=""; [ $2 != 0 ] && R=$2
  KFAC_X3_PAIR=$1 KFAC_SYRK_ROUNDS=$R timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_p$1_r$2.log 2>&1 || { tail -20 $O/alone_p$1_r$2.log; exit 1; }
  echo "pair$1 rounds$2: $(python -c "import json;d=json.loads(open('$O/alone_p$1_r$2.log').read().strip().splitlines()[-1]);print(round(d['x3_us_per_launch'],1), round(d['pass_ms'],4))")"
done
for cfg in "1 1" "0 0" "1 1" "0 0"; do
  set -- $cfg
  R=""; [ $2 != 0 ] && R=$2
  KFAC_X3_PAIR=$1 KFAC_SYRK_ROUNDS=$R timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-serial > $O/bench_p$1_r$2.log 2>&1 || { tail -20 $O/bench_p$1_r$2.log; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_p$1_r$2.log').read().strip().splitlines()[-1]);print('bench pair$1 rounds$2', round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['roofline']['avg_launch_us'],1), round(d['roofline']['frac'],3))"
done
