set -o pipefail
(cd tools/microbench && timeout -k 10 60 ./syrk_mb) && timeout -k 10 600 python -m pytest tests -m gpu -x -q 2>&1 | tail -5 && timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1; tail -2 gpurun_out/bench.log
