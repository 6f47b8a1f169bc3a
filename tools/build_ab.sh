#!/bin/bash
# Timing A/B builds of libkfac_hip.so into ab_libs/<name>/ (git-ignored; they travel to
# the GPU box with the tree): bash tools/build_ab.sh NAME -DMACRO=VALUE ...
# Run with BNN_KFAC_AMD_LIB=ab_libs/NAME/libkfac_hip.so python bench.py ...
set -e
name=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
out=$ROOT/ab_libs/$name
mkdir -p $out/obj
cd $ROOT/bnn_kfac_amd/csrc
FLAGS="--offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -fvisibility=hidden -munsafe-fp-atomics"
for f in factor invert quadform eig sample efb tripack capi; do
  /opt/rocm/bin/hipcc $FLAGS "$@" -c $f.hip -o $out/obj/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $out/libkfac_hip.so $out/obj/*.o
rm -rf $out/obj
echo "built $out/libkfac_hip.so"
