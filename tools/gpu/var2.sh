set -o pipefail
timeout -k 10 600 python -m pytest tests/test_gpu_eig_variance.py -x -q -k per_sample 2>&1 | grep -E "^E |Error" | head -20
