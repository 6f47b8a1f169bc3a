# Round 5: refresh the MLP bench's rocprofv3 kernel stats and PMC passes on the final
# tree (same-row inversion pairs; the x3 kernel unchanged since r05final)
set -o pipefail
export TMPDIR=/tmp
bash profiles/collect.sh r05final2 || exit 1
