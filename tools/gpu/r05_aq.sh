# Round 5: refresh the committed PMC traffic of the C5 (wide, kfac_factor_syrk3 now split
# in the workgroup) and C3 (LeNet-5) bench launches: profiles/collect.sh per config
set -o pipefail
export TMPDIR=/tmp
BENCH="python3 bench.py --config wide --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-serial --no-other-configs" bash profiles/collect.sh r05_wide || exit 1
BENCH="python3 bench.py --config lenet --steps 5 --warmup 2 --no-cpu-baseline --no-e2e --no-serial --no-other-configs" bash profiles/collect.sh r05_lenet || exit 1
