# Round 3: multi-batch conv jobs -- conv parity (factors + C3) then the LeNet-5 line.
set -o pipefail
mkdir -p gpurun_out/r03c
timeout -k 10 400 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r03c/tests.log 2>&1 || { tail -40 gpurun_out/r03c/tests.log; exit 1; }
tail -1 gpurun_out/r03c/tests.log
timeout -k 10 300 python bench.py --config lenet --no-cpu-baseline --no-e2e > gpurun_out/r03c/bench_lenet.log 2>&1 || { tail -20 gpurun_out/r03c/bench_lenet.log; exit 1; }
python -c "
import json; d=json.loads(open('gpurun_out/r03c/bench_lenet.log').read().strip().splitlines()[-1]); b=d['breakdown']
print('lenet %.4g ms/step %.3f'%(d['value'], d['ms_per_step']), b, d['roofline']['frac'], d['roofline']['launches'])"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r03c/prof -o run -- python3 bench.py --config lenet --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/r03c/prof.log 2>&1 || exit 1
python tools/kstats.py gpurun_out/r03c/prof | head -14
