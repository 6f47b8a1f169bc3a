set -o pipefail
mkdir -p gpurun_out
(cd tools/microbench && timeout -k 10 120 ./conv_ab > ../../gpurun_out/conv_ab.log 2>&1) || { tail gpurun_out/conv_ab.log; exit 1; }
cat gpurun_out/conv_ab.log
