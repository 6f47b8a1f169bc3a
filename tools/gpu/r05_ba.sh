# Round 5: 64-tile fp64 GEMMs with the A rows read once per 8 k for all four blocks of a
# wave (gemm_row_strip): inversion tests, then the wide MLP (C5) HEAD build vs this tree,
# alternating, twice
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ba
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_invert.py tests/test_gpu_invert_graph.py tests/test_gpu_wide.py tests/test_gpu_golden_r02.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for v in head new; do
if [ $v = head ]; then L=ab_libs/inv_head/libkfac_hip.so; else L=bnn_kfac_amd/libkfac_hip.so; fi
BNN_KFAC_AMD_LIB=$L timeout -k 10 300 python bench.py --config wide --steps 10 --warmup 3 --no-cpu-baseline --no-e2e > $O/wide_${v}_$r.log 2>&1 || { tail -20 $O/wide_${v}_$r.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/wide_${v}_$r.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('wide $v $r', round(d['value']/1e6,4), 'e6', round(d['ms_per_step'],3), 'ms serial', round(d['serial_images_per_s']/1e6,4), 'syrk', round(b['factor_tiles_ms_per_step'],3), 'inv', round(b['invert_ms_per_step'],3))"
done
done
