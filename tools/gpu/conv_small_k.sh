set -o pipefail
mkdir -p gpurun_out
cd tools/microbench
for k in 1 2 4 8 16; do
  KFAC_CONV_K=$k timeout -k 10 60 ./conv_ab 1 > ../../gpurun_out/csk$k.log 2>&1 || { cat ../../gpurun_out/csk$k.log; exit 1; }
  echo "k=$k $(grep 'us  (' ../../gpurun_out/csk$k.log | cut -c1-110)"
done
