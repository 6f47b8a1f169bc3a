# Round 4: register-prefetched bulk inversion updates (inv_bulk / inv_inner Z tiles):
# inversion parity, then wide step split and bench against the previous build (ab_libs/inv0)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04af
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_invert.py tests/test_gpu_invert_graph.py tests/test_gpu_wide.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "parity: $(tail -1 $O/tests.log)"
for lib in new inv0 new inv0; do
  L=bnn_kfac_amd/libkfac_hip.so; [ $lib = inv0 ] && L=ab_libs/inv0/libkfac_hip.so
  BNN_KFAC_AMD_LIB=$L timeout -k 10 200 python tools/step_split.py 8 wide > $O/split_$lib.log 2>&1 || { tail -20 $O/split_$lib.log; exit 1; }
  echo "== $lib split: $(grep -v amdgpu $O/split_$lib.log | tail -6 | tr '\n' ' ')"
done
for lib in new inv0; do
  L=bnn_kfac_amd/libkfac_hip.so; [ $lib = inv0 ] && L=ab_libs/inv0/libkfac_hip.so
  BNN_KFAC_AMD_LIB=$L timeout -k 10 300 python bench.py --config wide --steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-serial > $O/bench_$lib.log 2>&1 || { tail -20 $O/bench_$lib.log; exit 1; }
  echo "bench $lib: $(python -c "import json;d=json.loads(open('$O/bench_$lib.log').read().strip().splitlines()[-1]);print(d['value'], round(d['ms_per_step'],3), d['breakdown'])")"
done
