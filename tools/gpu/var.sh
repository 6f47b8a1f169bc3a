set -o pipefail
timeout -k 10 600 python -m pytest tests/test_gpu_eig_variance.py -x -q 2>&1 | tail -3 && timeout -k 10 600 python tools/bench_variance.py 2>&1 | tail -1
