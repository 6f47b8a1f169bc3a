# Round 5: wide C5 line, the split-in-workgroup SYRK planned with up to 4 (tree) or 16
# (s3r16) dispatch rounds; same box, alternating, twice
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ac
mkdir -p $O
for r in 1 2; do
for v in tree s3r16; do
if [ $v = tree ]; then unset BNN_KFAC_AMD_LIB; else export BNN_KFAC_AMD_LIB=$PWD/ab_libs/$v/libkfac_hip.so; fi
timeout -k 10 300 python bench.py --config wide --steps 10 --warmup 3 --no-cpu-baseline --no-e2e --no-serial > $O/wide_${v}_$r.log 2>&1 || { tail -20 $O/wide_${v}_$r.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/wide_${v}_$r.log').read().strip().splitlines()[-1])
print('$v $r', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['roofline']['launches'], d['breakdown'])"
done
done
