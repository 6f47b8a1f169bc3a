set -o pipefail
cd tools/microbench && timeout -k 10 120 ./diag_mb
