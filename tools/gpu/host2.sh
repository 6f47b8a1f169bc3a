set -o pipefail
timeout -k 10 300 python tools/host_overhead.py 2>&1 | grep -E "host issue|update\(\)"
