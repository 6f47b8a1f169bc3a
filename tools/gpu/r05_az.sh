# Round 5: the wide MLP (C5) with the inversion on 32-tiles (29 KB workgroups, which fit
# beside two kfac_factor_syrk3 workgroups per CU) instead of 64-tiles (70-107 KB, which
# do not), and the 4097^2 inversion alone on both; wide tests with 32-tiles forced
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05az
mkdir -p $O
KFAC_INV_TILE=32 timeout -k 10 600 python -u -m pytest tests/test_gpu_wide.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/wide_tests_t32.log 2>&1 || { tail -30 $O/wide_tests_t32.log; exit 1; }
tail -1 $O/wide_tests_t32.log
for r in 1 2; do
for t in 64 32; do
KFAC_INV_TILE=$t timeout -k 10 300 python bench.py --config wide --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $O/wide_t${t}_$r.log 2>&1 || { tail -20 $O/wide_t${t}_$r.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/wide_t${t}_$r.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('wide t$t $r', round(d['value']/1e6,4), 'e6', round(d['ms_per_step'],3), 'ms serial', round(d['serial_images_per_s']/1e6,4), 'syrk', round(b['factor_tiles_ms_per_step'],3), 'inv', round(b['invert_ms_per_step'],3))"
done
done
