# Round 5: KFAC.defer_bytes 256 vs 512 MiB on LeNet-5 (C3): the wide MLP's 281 MB updates stay one per launch at both
# caps; same box, alternating, twice
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ai
mkdir -p $O
for r in 1 2; do
for mb in 256 512; do
for c in lenet; do
timeout -k 10 300 python bench.py --config $c --steps 10 --warmup 3 --defer-mb $mb --no-cpu-baseline --no-e2e --no-serial > $O/${c}_${mb}_$r.log 2>&1 || { tail -20 $O/${c}_${mb}_$r.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/${c}_${mb}_$r.log').read().strip().splitlines()[-1])
print('$c $mb $r', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['launches'])"
done
done
done
