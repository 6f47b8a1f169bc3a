# A/B of environment knobs on the in-tree library (gpurun -- 'TAG=.. ENVS="a: b:KFAC_TILES_X3=1" CFG=lenet bash tools/gpu/ab_env.sh'):
# REPS alternating runs of the bench's pipelined loop per "name:VAR=value[,VAR=value]" (empty: defaults).
set -o pipefail
O=gpurun_out/${TAG:?set TAG}
mkdir -p $O
CFG=${CFG:-lenet}
ARGS=${ARGS:-"--steps 30 --warmup 5 --no-cpu-baseline --no-e2e --no-serial --no-other-configs --no-eig"}
for r in $(seq 1 ${REPS:-3}); do
  for v in $ENVS; do
    name=${v%%:*}; kv=${v#*:}
    env $(echo $kv | tr ',' ' ') timeout -k 10 300 python bench.py --config $CFG $ARGS > $O/ab_${CFG}_${name}_$r.log 2>&1 || { tail -20 $O/ab_${CFG}_${name}_$r.log; exit 1; }
    python -c "
import json; d=json.loads(open('$O/ab_${CFG}_${name}_$r.log').read().strip().splitlines()[-1])
print('$CFG $name rep $r', round(d['value']), round(d['ms_per_step'],4), json.dumps({k: round(v['ms_per_step'],4) for k,v in d['breakdown']['factor_kernels'].items()}))" | tee -a $O/ab_${CFG}.log
  done
done
