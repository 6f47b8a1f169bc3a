set -o pipefail
cd tools/microbench && timeout -k 10 60 ./syrk_mb 1024
