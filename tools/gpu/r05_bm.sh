# Round 5: 1-4 tasks per inversion workgroup (same-row chains reuse X[k][k] and C_i)
# vs HEAD (pairs) -- inversion tests at tpw 3 and 4, then inversion alone and MLP line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bm
mkdir -p $O
for t in 4 3 2; do
KFAC_INV_TPW=$t timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_invert.py tests/test_gpu_invert_graph.py tests/test_gpu_golden_r02.py tests/test_gpu_c2.py > $O/tests_$t.log 2>&1 || { tail -30 $O/tests_$t.log; exit 1; }
tail -1 $O/tests_$t.log
done
for r in 1 2; do
for v in head t2 t3 t4; do
  if [ $v = head ]; then L=ab_libs/inv_head/libkfac_hip.so; T=2; else L=bnn_kfac_amd/libkfac_hip.so; T=${v#t}; fi
  BNN_KFAC_AMD_LIB=$L KFAC_INV_TPW=$T timeout -k 10 120 python3 tools/probe_invert.py 300 $v >> $O/invert.log 2>&1 || { tail -5 $O/invert.log; exit 1; }
  BNN_KFAC_AMD_LIB=$L KFAC_INV_TPW=$T timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs > $O/b_${v}_$r.log 2>&1 || { tail -20 $O/b_${v}_$r.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/b_${v}_$r.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$v $r', d['value'], round(d['ms_per_step'],4), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4))"
done
done
grep median $O/invert.log
