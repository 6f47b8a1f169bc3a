# Round 5: two RCCL ranks on the one GPU of the box (rehearsal of the N > 1 path)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05aw
mkdir -p $O
timeout -k 10 120 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 tools/rccl_same_gpu.py > $O/rccl2.log 2>&1; echo "rc=$?"
tail -15 $O/rccl2.log
