set -o pipefail
mkdir -p gpurun_out
(cd tools/microbench && timeout -k 10 120 ./syrk_ab > ../../gpurun_out/syrk_ab.log 2>&1) || { tail gpurun_out/syrk_ab.log; exit 1; }
cat gpurun_out/syrk_ab.log
