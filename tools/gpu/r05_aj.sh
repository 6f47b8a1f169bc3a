# Round 5: where the pipelined MLP step's time goes after one launch per pass and the
# side-stream reduce: kernel trace of 200 steps (queues, gaps), the host/GPU step
# timeline, and a host profile of the bench loop
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aj
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-e2e --no-serial --no-other-configs > $O/trace.log 2>&1 || { tail -20 $O/trace.log; exit 1; }
python3 tools/trace_gaps.py $(ls $O/trace/*/run_kernel_trace.csv $O/trace/run_kernel_trace.csv 2>/dev/null | head -1) 20 > $O/gaps.txt 2>&1 || true
timeout -k 10 300 python3 tools/step_timeline.py 100 > $O/timeline.txt 2>&1 || { tail -20 $O/timeline.txt; exit 1; }
timeout -k 10 300 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-serial --no-other-configs --host-profile $O/host_profile.txt > $O/bench_hp.log 2>&1 || { tail -20 $O/bench_hp.log; exit 1; }
cat $O/gaps.txt | head -60
tail -30 $O/timeline.txt
head -45 $O/host_profile.txt
