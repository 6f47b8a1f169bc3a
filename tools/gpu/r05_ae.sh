# Round 5: the MNIST MLP line with every row-major launch on the split-in-workgroup
# kfac_factor_syrk3 (KFAC_SYRK3=1) against the default x3 kernel; same box, twice
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ae
mkdir -p $O
for r in 1 2; do
for v in x3 s3; do
if [ $v = s3 ]; then export KFAC_SYRK3=1; else unset KFAC_SYRK3; fi
timeout -k 10 300 python bench.py --steps 100 --warmup 10 --no-cpu-baseline --no-e2e --no-other-configs > $O/mlp_${v}_$r.log 2>&1 || { tail -20 $O/mlp_${v}_$r.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/mlp_${v}_$r.log').read().strip().splitlines()[-1])
print('$v $r', d['value'], d['ms_per_step'], d['roofline']['kernel'], d['roofline']['frac'], d['roofline']['avg_launch_us'], d['serial_images_per_s'])"
done
done
unset KFAC_SYRK3
