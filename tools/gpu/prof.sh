set -o pipefail
bash profiles/collect.sh r01
