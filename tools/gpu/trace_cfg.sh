# kernel trace (rocprofv3 --kernel-trace --stats) of one config's bench loop per library
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:?set TAG}
mkdir -p $O
for v in $AB; do
  name=${v%%:*}; dir=${v#*:}
  lib=$( [ "$dir" = "base" ] && echo bnn_kfac_amd/libkfac_hip.so || echo $dir/libkfac_hip.so )
  BNN_KFAC_AMD_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/tr_$name -o run -- python3 bench.py --config ${CFG:-lenet} --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-serial --no-eig > $O/tr_$name.log 2>&1 || { tail -20 $O/tr_$name.log; exit 1; }
  echo "== $name"; head -8 $O/tr_$name/run_kernel_stats.csv | cut -c1-150
done
