set -o pipefail
timeout -k 10 600 python tools/bench_variance.py 2>&1 | tail -2
