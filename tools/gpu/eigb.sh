set -o pipefail
timeout -k 10 300 python tools/bench_eig.py 129 785 2048 4097 2>&1 | tail -6
