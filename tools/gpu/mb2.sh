set -o pipefail
cd tools/microbench && for t in 512 1024 2048 3072; do timeout -k 10 60 ./syrk_mb $t || exit 1; done
