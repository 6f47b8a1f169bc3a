# Round 5: x3 task order inside each XCD's range (strided deal to the workgroups, so
# different tasks share a CU) vs the contiguous order -- C2 parity, then the MLP line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05bq
mkdir -p $O
for v in perm33 perm65; do
BNN_KFAC_AMD_LIB=ab_libs/$v/libkfac_hip.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_c2.py > $O/tests_$v.log 2>&1 || { tail -30 $O/tests_$v.log; exit 1; }
tail -1 $O/tests_$v.log
done
for r in 1 2 3; do
for v in head perm33 perm65; do
  if [ $v = head ]; then L=bnn_kfac_amd/libkfac_hip.so; else L=ab_libs/$v/libkfac_hip.so; fi
  BNN_KFAC_AMD_LIB=$L timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs --no-serial > $O/b_${v}_$r.log 2>&1 || { tail -20 $O/b_${v}_$r.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/b_${v}_$r.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$v $r', d['value'], round(d['ms_per_step'],4), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4))"
done
done
