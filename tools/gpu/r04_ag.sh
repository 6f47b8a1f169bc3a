# Round 4: panels per bulk inversion update (KFAC_INV_BLOCK) with the register-prefetched
# bulk updates, wide config step split
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ag
mkdir -p $O
for pb in 4 8 6 4 8; do
  KFAC_INV_BLOCK=$pb timeout -k 10 200 python tools/step_split.py 8 wide > $O/split_pb$pb.log 2>&1 || { tail -20 $O/split_pb$pb.log; exit 1; }
  echo "== PB $pb: $(grep -v amdgpu $O/split_pb$pb.log | tail -6 | tr '\n' ' ')"
done
