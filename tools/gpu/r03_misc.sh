# Round 3: bf16x3 SYRK (119-VGPR producer) parity with every row-major factor forced
# through it, wide / MLP lines, then the eigensolver's HBM counters at n = 4097
# (separate FETCH_SIZE / WRITE_SIZE passes, MI355X_MICROARCH.md).
set -o pipefail
mkdir -p gpurun_out/r03m
KFAC_SYRK3=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py tests/test_gpu_wide.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03m/tests_s3.log 2>&1 || { tail -40 gpurun_out/r03m/tests_s3.log; exit 1; }
tail -1 gpurun_out/r03m/tests_s3.log
timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e > gpurun_out/r03m/bench_wide.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/r03m/bench_mlp.log 2>&1 || exit 1
KFAC_SYRK3=1 timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/r03m/bench_mlp_s3.log 2>&1 || exit 1
for f in bench_wide bench_mlp bench_mlp_s3; do python -c "
import json,sys; d=json.loads(open('gpurun_out/r03m/$f.log').read().strip().splitlines()[-1]); b=d['breakdown']
print('$f', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], d['roofline']['kernel'], 'frac %.3f'%d['roofline']['frac'])"; done
export TMPDIR=/tmp
for C in FETCH_SIZE WRITE_SIZE; do
  EIG_NO_CPU=1 timeout -k 10 200 rocprofv3 --pmc $C --kernel-include-regex "eig_" --output-format csv -d gpurun_out/r03m/eig_$C -o run -- python3 tools/bench_eig.py 4097 > gpurun_out/r03m/eig_$C.log 2>&1
  rc=$?; echo "eig pmc $C rc=$rc"; [ $rc -le 2 ] || exit $rc
done
EIG_NO_CPU=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03m/eig_trace -o run -- python3 tools/bench_eig.py 4097 > gpurun_out/r03m/eig_trace.log 2>&1 || exit 1
