#!/bin/bash
# Build in-tree (so the snapshot carries a fresh libkfac_hip.so), then run a script on the GPU box.
set -e
cd "$(dirname "$0")/.."
make -C bnn_kfac_amd/csrc -j8 > /dev/null
exec /usr/local/graft/bin/gpurun --timeout "${GPU_TIMEOUT:-900}" -- "bash $1"
