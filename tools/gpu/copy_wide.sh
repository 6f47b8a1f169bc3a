# (1) conv parity with the mode-3 image copy (default), LeNet-5 lines copy vs
# KFAC_CONV_COPY=0 and a kernel trace; (2) wide MLP: x3 SYRK vs split-pass syrk3
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/cw
timeout -k 10 400 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py tests/test_gpu_golden_r02.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/cw/tests.log 2>&1 || { tail -40 gpurun_out/cw/tests.log; exit 1; }
tail -1 gpurun_out/cw/tests.log
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']; r=d['roofline']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'inv %.3f'%b['invert_ms_per_step'], r['kernel'], 'avg_us %.1f'%r['avg_launch_us'], 'frac %.3f'%r['frac'], 'serial %.4g'%(d.get('serial_images_per_s') or 0))"; }
for r in 1 2; do
  timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/cw/lenet_copy_$r.log 2>&1 || exit 1
  show gpurun_out/cw/lenet_copy_$r.log
  KFAC_CONV_COPY=0 timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/cw/lenet_nocopy_$r.log 2>&1 || exit 1
  show gpurun_out/cw/lenet_nocopy_$r.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cw/trace_copy -o run -- python3 bench.py --config lenet --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/cw/trace_copy.log 2>&1 || exit 1
head -8 gpurun_out/cw/trace_copy/run_kernel_stats.csv | cut -c1-150
timeout -k 10 -s KILL 120 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT --kernel-include-regex "kfac_factor_conv" --output-format csv -d gpurun_out/cw/pmc_lds -o run -- python3 bench.py --config lenet --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/cw/pmc_lds.log 2>&1; echo "pmc rc=$?"
for r in 1 2; do
  KFAC_SYRK3=0 KFAC_TILES_X3=1 timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/cw/wide_x3_$r.log 2>&1 || exit 1
  show gpurun_out/cw/wide_x3_$r.log
  timeout -k 10 300 python bench.py --config wide --no-cpu-baseline --no-e2e --steps 20 > gpurun_out/cw/wide_d_$r.log 2>&1 || exit 1
  show gpurun_out/cw/wide_d_$r.log
done
