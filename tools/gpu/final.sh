set -o pipefail
timeout -k 10 900 bash profiles/collect.sh r01 && timeout -k 10 600 python bench.py > gpurun_out/bench_full.log 2>&1; tail -1 gpurun_out/bench_full.log
