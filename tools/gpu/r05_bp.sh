# Round 5: look-ahead of the blocked (wide) inversion -- the rest of each block's bulk
# update on a helper stream beside the next block's panel chain.  Wide / large-size
# inversion tests first, then the wide inversion alone and C5, look-ahead on vs off
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bp
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_invert.py tests/test_gpu_invert_graph.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for la in 1 0; do
  KFAC_INV_LOOKAHEAD=$la timeout -k 10 200 python3 tools/probe_invert.py 20 la$la wide >> $O/invert.log 2>&1 || { tail -5 $O/invert.log; exit 1; }
done
done
grep median $O/invert.log
for r in 1 2; do
for la in 1 0; do
  KFAC_INV_LOOKAHEAD=$la timeout -k 10 300 python3 bench.py --config wide --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $O/wide_la${la}_$r.log 2>&1 || { tail -20 $O/wide_la${la}_$r.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/wide_la${la}_$r.log').read().strip().splitlines()[-1])
print('la$la $r', d['value'], round(d['ms_per_step'],3), 'serial', d.get('serial_images_per_s'), d['breakdown'])"
done
done
