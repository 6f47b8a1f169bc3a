set -o pipefail
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/gpu_tests.log 2>&1; rc=$?; tail -3 gpurun_out/gpu_tests.log; [ $rc -eq 0 ] && \
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/bench.log 2>&1 && \
python -c "import json; d=json.loads(open('gpurun_out/bench.log').read().strip().splitlines()[-1]); print(d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['breakdown'])"
