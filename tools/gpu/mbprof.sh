set -o pipefail
export TMPDIR=/tmp
root=$PWD
cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $root/gpurun_out/mbprof -o mb -- $root/tools/microbench/syrk_mb 1024 > $root/gpurun_out/mbprof.log 2>&1
cd $root && python tools/kstats.py gpurun_out/mbprof
