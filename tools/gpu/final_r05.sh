# Round 5 end check: the whole GPU suite, the factor suites with every row-major launch
# forced through kfac_factor_syrk3, smoke, the bench as the driver runs it
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r05_end4}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -2 $O/gpu_tests.log
KFAC_SYRK3=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_factors.py tests/test_gpu_ragged.py tests/test_gpu_c2.py tests/test_gpu_golden_r02.py -m gpu -k "not x3_ and not test_queued_pass_matches" > $O/forced_syrk3_tests.log 2>&1 || { tail -30 $O/forced_syrk3_tests.log; exit 1; }
tail -1 $O/forced_syrk3_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_mlp.log 2>&1 || { tail -20 $O/bench_mlp.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench_mlp.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['serial_images_per_s'], d['breakdown'])
for k,v in d['other_configs'].items(): print(k, v['value'], v['ms_per_step'], v['roofline']['kernel'], v['roofline']['frac'])"
