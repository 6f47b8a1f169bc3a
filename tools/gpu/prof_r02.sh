# Round-2 profiles: rocprofv3 kernel stats + PMC passes for the MLP (default), wide and
# LeNet-5 bench lines (profiles/collect.sh recipe), plus one full bench line per config.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --config wide > gpurun_out/bench_wide.log 2>&1 || { tail -5 gpurun_out/bench_wide.log; exit 1; }
timeout -k 10 300 python bench.py --config lenet > gpurun_out/bench_lenet.log 2>&1 || { tail -5 gpurun_out/bench_lenet.log; exit 1; }
bash profiles/collect.sh r02 || exit 1
BENCH="python3 bench.py --config wide --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-serial" bash profiles/collect.sh r02_wide || exit 1
BENCH="python3 bench.py --config lenet --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-serial" bash profiles/collect.sh r02_lenet || exit 1
