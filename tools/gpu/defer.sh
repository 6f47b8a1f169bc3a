set -o pipefail
(cd tools/microbench && timeout -k 10 60 ./syrk_mb 1024) && \
timeout -k 10 600 python -m pytest tests/test_gpu_factors.py tests/test_gpu_distributed.py -x -q > gpurun_out/defer_tests.log 2>&1; tail -3 gpurun_out/defer_tests.log && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench.log 2>&1 && \
python -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['breakdown'])"
