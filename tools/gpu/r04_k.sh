# Round 4: x3 accumulators pinned in AGPRs (A/B: parity + SYRK alone + bench)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
A=ab_libs/agpr/libkfac_hip.so
BNN_KFAC_AMD_LIB=$A timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py -x -q --timeout 200 --timeout-method thread > $O/agpr_tests.log 2>&1 || { tail -30 $O/agpr_tests.log; exit 1; }
echo "agpr parity: $(tail -1 $O/agpr_tests.log)"
timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_def.log 2>&1 || { tail -20 $O/alone_def.log; exit 1; }
BNN_KFAC_AMD_LIB=$A timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_agpr.log 2>&1 || { tail -20 $O/alone_agpr.log; exit 1; }
echo "alone def: $(tail -1 $O/alone_def.log)"
echo "alone agpr: $(tail -1 $O/alone_agpr.log)"
