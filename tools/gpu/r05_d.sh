# Round 5: 16x16x32 parts-in-K CU-tile variants; the C2 bench-pass oracle test and the
# invert tests (fresh verdict tensors); the bench line with its C3 / C5 legs; last, the
# exit-time SIGSEGV probe with /proc/self/maps (expected to end in 139: nothing after it)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05d
mkdir -p $O
timeout -k 10 120 ./tools/microbench/cut_mb > $O/cut_mb.log 2>&1; echo "cut_mb rc $?"; cat $O/cut_mb.log
timeout -k 10 600 python -u -m pytest tests/test_gpu_c2.py tests/test_gpu_invert_graph.py tests/test_gpu_invert.py tests/test_gpu_boundary.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
tail -1 $O/tests.log
/usr/bin/time -v timeout -k 10 400 python bench.py > $O/bench_mlp.log 2> $O/bench_time.log || { tail -20 $O/bench_mlp.log $O/bench_time.log; exit 1; }
grep -E "Elapsed|Maximum resident" $O/bench_time.log
python -c "
import json;d=json.loads(open('$O/bench_mlp.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['serial_images_per_s'])
for k,v in d['other_configs'].items(): print(k, v['value'], v['ms_per_step'], v['roofline']['kernel'], v['roofline']['frac'])"
cd /tmp && EXIT_MAPS=$GRAFT_REPO_ROOT/$O/exit_maps.txt timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$O/prof_exit -- python3 $GRAFT_REPO_ROOT/tools/exit_probe.py eig > $GRAFT_REPO_ROOT/$O/exit_eig.log 2>&1; echo "exit probe rc $?"
