# Round 4, second run: the wave-tile / prefetch microbench variants and the exit-time
# SIGSEGV bisection under rocprofv3 --pmc (tools/exit_probe.py), plus a host-side cProfile
# of the bench's pipelined step.
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
timeout -k 10 120 ./tools/microbench/x3w_mb > $O/x3w_mb.log 2>&1; echo "x3w_mb rc $?"; cat $O/x3w_mb.log
timeout -k 10 300 python bench.py --steps 30 --no-cpu-baseline --no-e2e --no-serial --host-profile $O/host_profile.txt > $O/bench_hp.log 2>&1 || { tail -20 $O/bench_hp.log; exit 1; }
head -1 $O/host_profile.txt
cd /tmp
for m in load factor eig eig_os; do
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d $GRAFT_REPO_ROOT/$O/exit_$m -o run -- python3 $GRAFT_REPO_ROOT/tools/exit_probe.py $m > $GRAFT_REPO_ROOT/$O/exit_$m.log 2>&1; echo "exit probe $m under pmc: rc $?"
done
exit 0
