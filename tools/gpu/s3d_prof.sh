# kernel stats of the pre-split bf16x3 path (KFAC_SYRK3=2): wide and MLP
set -o pipefail
mkdir -p gpurun_out/s3dp
export TMPDIR=/tmp
for C in wide mlp; do
  KFAC_SYRK3=2 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/s3dp/$C -o run -- python3 bench.py --config $C --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/s3dp/$C.log 2>&1 || exit 1
  python tools/kstats.py gpurun_out/s3dp/$C | head -8
done
