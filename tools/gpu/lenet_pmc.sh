# LeNet-5 PMC passes (conv kernels): where the staged conv kernel's time goes
set -o pipefail
BENCH="python3 bench.py --config lenet --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-serial" bash profiles/collect.sh r03_lenet_pmc > gpurun_out/prof_r03_lenet_pmc.log 2>&1 || { tail -20 gpurun_out/prof_r03_lenet_pmc.log; exit 1; }
tail -8 gpurun_out/prof_r03_lenet_pmc.log
