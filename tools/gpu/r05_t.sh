# Round 5: select-free 16-column elimination with a v_rcp_f64 + Newton reciprocal (no
# SGPR spills): invert parity, the bench, and the inversion's kernel times
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05t
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_invert.py tests/test_gpu_invert_graph.py tests/test_gpu_c2.py tests/test_gpu_golden_r02.py tests/test_gpu_eig_variance.py -m gpu > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-e2e > $O/bench.log 2>&1 || { tail -20 $O/bench.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/bench.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['serial_images_per_s'], d['breakdown'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o run -- python3 bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-e2e --no-other-configs > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
grep -E "inv_step|x3|reduce|copy_out" $O/trace/run_kernel_stats.csv | cut -d, -f1-4
