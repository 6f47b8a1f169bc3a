# Round 5: kfac_factor_syrk3 with the split made in the workgroup (no split pass): the
# wide tests, the factor / C3 / C2 suites with every row-major launch forced through it
# (KFAC_SYRK3=1), then the bench line (C5 in other_configs) and the kernel trace of C5
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ad
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_wide.py -m gpu > $O/wide_tests.log 2>&1 || { tail -30 $O/wide_tests.log; exit 1; }
tail -1 $O/wide_tests.log
KFAC_SYRK3=1 timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_factors.py tests/test_gpu_ragged.py tests/test_gpu_c2.py tests/test_gpu_golden_r02.py -m gpu -k "not x3_ and not test_queued_pass_matches" > $O/forced_tests.log 2>&1 || { tail -30 $O/forced_tests.log; exit 1; }
tail -1 $O/forced_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['serial_images_per_s'])
for k,v in d['other_configs'].items(): print(k, v['value'], v['ms_per_step'], v['roofline']['kernel'], v['roofline']['frac'], v['roofline']['avg_launch_us'], v['breakdown'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --config wide --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-serial > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep -E "syrk3|split3|inv_|reduce" $O/trace/run_kernel_stats.csv | cut -d, -f1-4
