# Round 4: host cost of the C-ABI calls of an MLP step (graph-launched and plain inversion)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
timeout -k 10 200 python tools/host_api_bench.py 200 > $O/host_api.log 2>&1 || { tail -20 $O/host_api.log; exit 1; }
echo "graph: $(tail -1 $O/host_api.log)"
KFAC_INV_GRAPH=0 timeout -k 10 200 python tools/host_api_bench.py 200 > $O/host_api_nograph.log 2>&1 || { tail -20 $O/host_api_nograph.log; exit 1; }
echo "nograph: $(tail -1 $O/host_api_nograph.log)"
