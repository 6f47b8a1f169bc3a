set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_invert.py tests/test_gpu_eig_variance.py tests/test_gpu_distributed.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gpu_inv.log 2>&1; rc=$?
tail -2 gpurun_out/gpu_inv.log; [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" gpurun_out/gpu_inv.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench.log 2>&1 || exit $?
python -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['roofline']['frac'], d['breakdown'])"
bash tools/gpu/trace_gaps.sh
