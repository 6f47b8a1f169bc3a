set -o pipefail
timeout -k 10 300 python tools/bench_factor_jobs.py lenet 2>&1 | grep -v UserWarn | tail -8
