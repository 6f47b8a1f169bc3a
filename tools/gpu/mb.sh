set -o pipefail
cd tools/microbench && timeout -k 10 120 ./syrk_mb 1024 && timeout -k 10 120 ./syrk_mb 1024
