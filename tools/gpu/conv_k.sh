set -o pipefail
mkdir -p gpurun_out
for k in 1 2 3 4 8; do
  (cd tools/microbench && KFAC_CONV_K=$k timeout -k 10 120 ./conv_ab > ../../gpurun_out/conv_k$k.log 2>&1) || { tail gpurun_out/conv_k$k.log; exit 1; }
  echo "K=$k"; grep "us  (" gpurun_out/conv_k$k.log | cut -c1-80
done
