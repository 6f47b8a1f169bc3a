# Round 5: panels per blocked update (KFAC_INV_BLOCK) with the look-ahead and the
# 16-byte loads: 4 (default) vs 6 vs 8 -- wide inversion alone and C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bw
mkdir -p $O
KFAC_INV_BLOCK=8 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wide.py > $O/tests_b8.log 2>&1 || { tail -30 $O/tests_b8.log; exit 1; }
tail -1 $O/tests_b8.log
for r in 1 2; do
for b in 4 6 8; do
  KFAC_INV_BLOCK=$b timeout -k 10 200 python3 tools/probe_invert.py 20 wide_b$b wide >> $O/invert.log 2>&1 || { tail -5 $O/invert.log; exit 1; }
done
done
grep median $O/invert.log
for b in 4 6 8; do
  KFAC_INV_BLOCK=$b timeout -k 10 300 python3 bench.py --config wide --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-serial > $O/wide_b$b.log 2>&1 || { tail -20 $O/wide_b$b.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/wide_b$b.log').read().strip().splitlines()[-1])
print('b$b', d['value'], round(d['ms_per_step'],3))"
done
