# Round 5: GPU suite with the ragged last batch; the bench line (with C3 / C5); last,
# the exit-time SIGSEGV probe with /proc/self/maps (expected 139: nothing after it)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05g
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
S=$(date +%s)
timeout -k 10 400 python bench.py > $O/bench_mlp.log 2>&1 || { tail -20 $O/bench_mlp.log; exit 1; }
echo "bench wall $(( $(date +%s) - S )) s"
python -c "
import json;d=json.loads(open('$O/bench_mlp.log').read().strip().splitlines()[-1])
print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['serial_images_per_s'], d['breakdown'])
for k,v in d['other_configs'].items(): print(k, v['value'], v['ms_per_step'], v['roofline']['kernel'], v['roofline']['frac'], v['breakdown'])"
cd /tmp && EXIT_MAPS=$GRAFT_REPO_ROOT/$O/exit_maps.txt timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$O/prof_exit -- python3 $GRAFT_REPO_ROOT/tools/exit_probe.py eig > $GRAFT_REPO_ROOT/$O/exit_eig.log 2>&1; echo "exit probe rc $?"
