set -o pipefail
EIG_VECS=1 timeout -k 10 300 python tools/bench_eig.py 300 785 2048 2>&1 | grep -v amdgpu && timeout -k 10 600 python -m pytest tests/test_gpu_eig_variance.py -x -q 2>&1 | tail -2
