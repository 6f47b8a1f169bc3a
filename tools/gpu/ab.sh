set -o pipefail
cd _head && timeout -k 10 200 python tools/probe_defer.py mlp 2>&1 | grep defer_batches && cd .. && timeout -k 10 200 python tools/probe_defer.py mlp 2>&1 | grep defer_batches
