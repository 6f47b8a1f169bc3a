# Round 5: KFAC.defer_bytes 256 vs 512 MiB on the wide MLP (C5): at 512 MiB two 281 MB
# updates queue per launch (562 MB >= the cap), at 256 one; same box, alternating, twice
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05ar
mkdir -p $O
for r in 1 2; do
for mb in 256 512; do
timeout -k 10 300 python bench.py --config wide --steps 10 --warmup 3 --defer-mb $mb --no-cpu-baseline --no-e2e --no-serial > $O/wide_${mb}_$r.log 2>&1 || { tail -20 $O/wide_${mb}_$r.log; exit 1; }
python -c "
import json;d=json.loads(open('$O/wide_${mb}_$r.log').read().strip().splitlines()[-1])
print('wide $mb $r', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['launches'], d['breakdown'])"
done
done
