# Round 5: 16-byte tile stores and LDS-staged wide read-modify-writes in the blocked
# inversion kernels vs HEAD (16-byte loads) -- tests, inversions alone, MLP line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bv
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_invert.py tests/test_gpu_invert_graph.py tests/test_gpu_golden_r02.py tests/test_gpu_c2.py tests/test_gpu_wide.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for v in head new; do
  if [ $v = head ]; then L=ab_libs/inv_head/libkfac_hip.so; else L=bnn_kfac_amd/libkfac_hip.so; fi
  BNN_KFAC_AMD_LIB=$L timeout -k 10 120 python3 tools/probe_invert.py 300 $v >> $O/invert.log 2>&1 || { tail -5 $O/invert.log; exit 1; }
  BNN_KFAC_AMD_LIB=$L timeout -k 10 200 python3 tools/probe_invert.py 20 wide_$v wide >> $O/invert.log 2>&1 || { tail -5 $O/invert.log; exit 1; }
  BNN_KFAC_AMD_LIB=$L timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs --no-serial > $O/b_${v}_$r.log 2>&1 || { tail -20 $O/b_${v}_$r.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/b_${v}_$r.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$v $r', d['value'], round(d['ms_per_step'],4), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4))"
done
done
grep median $O/invert.log
