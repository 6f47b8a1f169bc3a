# Round 5: 16-byte conflict-free fp64 MFMA operand reads (NB + 4 pitch) in the
# inversion: same-box A/B against the committed build (inv_head) -- the MLP inversion
# alone and the wide C5 line -- then the inversion parity suites
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05af
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_invert.py tests/test_gpu_invert_graph.py tests/test_gpu_wide.py tests/test_gpu_golden_r02.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do
for v in head tree; do
if [ $v = tree ]; then unset BNN_KFAC_AMD_LIB; else export BNN_KFAC_AMD_LIB=$PWD/ab_libs/inv_$v/libkfac_hip.so; fi
timeout -k 10 200 python tools/probe_invert.py 300 $v >> $O/inv.log 2>&1 || { tail -20 $O/inv.log; exit 1; }
timeout -k 10 300 python bench.py --config wide --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-serial > $O/wide_${v}_$r.log 2>&1 || { tail -20 $O/wide_${v}_$r.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/wide_${v}_$r.log').read().strip().splitlines()[-1])
print('$v $r', d['value'], d['ms_per_step'], d['breakdown'])"
done
done
unset BNN_KFAC_AMD_LIB
grep median $O/inv.log
