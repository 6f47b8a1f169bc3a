# Round 5: KFAC.defer_bytes 256 MiB (default) vs 1 GiB on LeNet-5 (C3) and the wide MLP
# (C5) now that the wide SYRK has no split images; same box, alternating, twice
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ah
mkdir -p $O
for r in 1 2; do
for mb in 256 1024; do
for c in lenet wide; do
timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --defer-mb $mb --no-cpu-baseline --no-e2e --no-serial > $O/${c}_${mb}_$r.log 2>&1 || { tail -20 $O/${c}_${mb}_$r.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/${c}_${mb}_$r.log').read().strip().splitlines()[-1])
print('$c $mb $r', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['launches'])"
done
done
done
