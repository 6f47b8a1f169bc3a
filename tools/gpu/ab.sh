# A/B of prebuilt library variants on one box (gpurun -- 'TAG=.. AB="base:ab_libs/x" CFG=mlp bash tools/gpu/ab.sh'):
# REPS alternating runs of the bench's pipelined loop per variant ("name:libdir", the
# in-tree library for "base"), one JSON line each into gpurun_out/$TAG/ab_<cfg>.log.
set -o pipefail
O=gpurun_out/${TAG:?set TAG}
mkdir -p $O
CFG=${CFG:-mlp}
ARGS=${ARGS:-"--steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-serial --no-other-configs --no-eig"}
for r in $(seq 1 ${REPS:-3}); do
  for v in $AB; do
    name=${v%%:*}; dir=${v#*:}
    lib=$( [ "$dir" = "base" ] && echo bnn_kfac_amd/libkfac_hip.so || echo $dir/libkfac_hip.so )
    BNN_KFAC_AMD_LIB=$lib timeout -k 10 300 python bench.py --config $CFG $ARGS > $O/ab_${CFG}_${name}_$r.log 2>&1 || { tail -20 $O/ab_${CFG}_${name}_$r.log; exit 1; }
    python -c "
import json,sys; d=json.loads(open('$O/ab_${CFG}_${name}_$r.log').read().strip().splitlines()[-1]); r=d['roofline']
print('$CFG $name rep $r', round(d['value']), round(d['ms_per_step'],4), r['kernel'], round(r['avg_launch_us'],1), round(r['frac'],4), json.dumps({k: round(v['ms_per_step'],4) for k,v in d['breakdown']['factor_kernels'].items()}))" | tee -a $O/ab_${CFG}.log
  done
done
