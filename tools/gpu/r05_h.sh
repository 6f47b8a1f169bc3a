# Round 5: ragged last batch without the argument-block scratch copy: its tests, the
# bench line, and LeNet-5 on the current library vs HEAD's (ab_libs/head) to place the
# C3 slowdown seen in the first other_configs line
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05h
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_ragged.py tests/test_gpu_c2.py tests/test_gpu_factors.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
timeout -k 10 400 python bench.py --no-cpu-baseline --no-e2e > $O/bench_mlp.log 2>&1 || { tail -20 $O/bench_mlp.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench_mlp.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['serial_images_per_s'], d['breakdown'])
for k,v in d['other_configs'].items(): print(k, v['value'], v['ms_per_step'], v['roofline']['kernel'], v['roofline']['frac'], v['breakdown'])"
for L in head cur; do
  if [ $L = head ]; then export BNN_KFAC_AMD_LIB=$PWD/ab_libs/head/libkfac_hip.so; else unset BNN_KFAC_AMD_LIB; fi
  timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e --no-serial > $O/bench_lenet_$L.log 2>&1 || { tail -20 $O/bench_lenet_$L.log; exit 1; }
  python -c "
import json;d=json.loads(open('$O/bench_lenet_$L.log').read().strip().splitlines()[-1])
print('$L lenet', d['value'], d['ms_per_step'], d['roofline']['frac'], d['breakdown'])"
done
