set -o pipefail
R=$PWD; cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tr -o run -- python3 $R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > $R/gpurun_out/tr.log 2>&1
cut -c1-150 $R/gpurun_out/tr/run_kernel_stats.csv | head -12
