# kfac_factor_conv_x3: conv parity tests, then the LeNet-5 (C3) line with / without it
set -o pipefail
O=gpurun_out/${TAG:?set TAG}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_factors.py tests/test_gpu_c3.py -m gpu -k "conv or c3 or lenet or hooks" > $O/conv_tests.log 2>&1 || { tail -40 $O/conv_tests.log; exit 1; }
tail -2 $O/conv_tests.log
for r in 1 2 3; do
  for x in 1 0; do
    KFAC_CONV_X3=$x timeout -k 10 300 python bench.py --config lenet --steps 30 --warmup 5 --no-cpu-baseline --no-e2e --no-serial --no-eig > $O/lenet_x3_${x}_$r.log 2>&1 || { tail -20 $O/lenet_x3_${x}_$r.log; exit 1; }
    python -c "
import json; d=json.loads(open('$O/lenet_x3_${x}_$r.log').read().strip().splitlines()[-1]); r=d['roofline']
print('conv_x3=$x rep $r', round(d['value']), round(d['ms_per_step'],4), r['kernel'], round(r['avg_launch_us'],1), round(r['frac'],4), json.dumps({k: (round(v['ms_per_step'],4), round(v['tflops'] or 0,1)) for k,v in d['breakdown']['factor_kernels'].items()}))" | tee -a $O/ab_lenet.log
  done
done
