set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_efb.py -x -v --timeout 120 --timeout-method thread > gpurun_out/gpu_efb.log 2>&1 || { tail -60 gpurun_out/gpu_efb.log; exit 1; }
tail -3 gpurun_out/gpu_efb.log
