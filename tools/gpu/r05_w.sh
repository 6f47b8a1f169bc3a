# Round 5: Y-row dummy slots without bank conflicts -- same-box A/B against the
# committed elimination (inv_head), then the LDS counters of inv_step
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05w
mkdir -p $O
for r in 1 2; do
for v in head tree; do
if [ $v = tree ]; then unset BNN_KFAC_AMD_LIB; else export BNN_KFAC_AMD_LIB=$PWD/ab_libs/inv_$v/libkfac_hip.so; fi
timeout -k 10 200 python tools/probe_invert.py 300 $v >> $O/ab.log 2>&1 || { tail -20 $O/ab.log; exit 1; }
done
done
unset BNN_KFAC_AMD_LIB
grep median $O/ab.log
timeout -k 10 120 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_invert.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES --kernel-include-regex "inv_step" --output-format csv -d $O/pmc -o run -- python3 tools/probe_invert.py 50 pmc > $O/pmc.log 2>&1
echo "pmc rc=$?"
