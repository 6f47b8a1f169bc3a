# grouped MLP inversion alone: single steps vs pairs, tasks per workgroup 2 / 1;
# kernel trace of both chains
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pp
for P in 0 1; do for W in 2 1; do
  KFAC_INV_PAIR=$P KFAC_INV_TPW=$W timeout -k 10 120 python tools/probe_pair.py 300 || exit 1
done; done
for P in 0 1; do
  KFAC_INV_PAIR=$P timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pp/trace_$P -o run -- python3 tools/probe_pair.py 50 > gpurun_out/pp/trace_$P.log 2>&1 || exit 1
  head -8 gpurun_out/pp/trace_$P/run_kernel_stats.csv | cut -c1-160
done
