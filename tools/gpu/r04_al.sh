# Round 4: wave priority of the wide inversion's two-launch steps (KFAC_INV_BLK_PRIO)
# beside the pass: the inversion is the wide step's critical path
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04al
mkdir -p $O
KFAC_INV_BLK_PRIO=3 timeout -k 10 600 python -u -m pytest tests/test_gpu_invert.py tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "parity (prio 3): $(tail -1 $O/tests.log)"
for p in 0 3 0 3 2; do
  KFAC_INV_BLK_PRIO=$p timeout -k 10 300 python bench.py --config wide --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-serial > $O/bench_p$p.log 2>&1 || { tail -20 $O/bench_p$p.log; exit 1; }
  echo "prio $p: $(python -c "import json;d=json.loads(open('$O/bench_p$p.log').read().strip().splitlines()[-1]);b=d['breakdown'];print(round(d['value']/1e6,4), round(d['ms_per_step'],3), round(b['factor_tiles_ms_per_step'],3), round(b['invert_ms_per_step'],3))")"
done
