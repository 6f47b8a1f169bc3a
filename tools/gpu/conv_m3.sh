# conv factors with 17..32 columns: three 16x16x4 blocks (default) vs one 32x32 block
set -o pipefail
mkdir -p gpurun_out/m3
timeout -k 10 400 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/m3/tests.log 2>&1 || { tail -40 gpurun_out/m3/tests.log; exit 1; }
tail -1 gpurun_out/m3/tests.log
show() { python -c "
import json; d=json.loads(open('$1').read().strip().splitlines()[-1]); b=d['breakdown']
print('$1', '%.4g'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f'%b['factor_tiles_ms_per_step'], 'frac %.3f'%d['roofline']['frac'], 'host %.3f'%b['host_issue_ms_per_step'])"; }
for L in m3 o3; do
  LIB=$PWD/bnn_kfac_amd/libkfac_hip.so; [ $L = o3 ] && LIB=$PWD/bnn_kfac_amd/libkfac_hip_o3.so
  BNN_KFAC_AMD_LIB=$LIB timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --no-serial --steps 20 > gpurun_out/m3/lenet_$L.log 2>&1 || exit 1
  show gpurun_out/m3/lenet_$L.log
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/m3/prof -o run -- python3 bench.py --config lenet --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/m3/prof.log 2>&1 || exit 1
python tools/kstats.py gpurun_out/m3/prof > gpurun_out/m3/kstats.txt; head -7 gpurun_out/m3/kstats.txt
