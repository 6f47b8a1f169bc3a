# Round 5: rocprofv3 kernel stats + PMC passes of the predictive-variance path
# (tools/bench_variance.py: kfac_kron_quadform), the first since round 1
set -o pipefail
export TMPDIR=/tmp
BENCH="python3 tools/bench_variance.py" bash profiles/collect.sh r05_quad || exit 1
timeout -k 10 300 python3 tools/bench_variance.py > gpurun_out/prof_r05_quad/variance.json 2>&1 || exit 1
tail -1 gpurun_out/prof_r05_quad/variance.json
