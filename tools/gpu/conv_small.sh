set -o pipefail
mkdir -p gpurun_out
cd tools/microbench
for s in 0 1; do
  KFAC_CONV_SMALL=$s timeout -k 10 60 ./conv_ab 1 > ../../gpurun_out/cs$s.log 2>&1 || { cat ../../gpurun_out/cs$s.log; exit 1; }
  KFAC_CONV_SMALL=$s timeout -k 10 60 ./conv_ab 3 >> ../../gpurun_out/cs$s.log 2>&1 || { cat ../../gpurun_out/cs$s.log; exit 1; }
  echo "small=$s"; grep "us  (" ../../gpurun_out/cs$s.log
done
