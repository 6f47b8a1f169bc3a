set -o pipefail
mkdir -p gpurun_out
for r in 1 2 3 4; do
  (cd tools/microbench && KFAC_SYRK_ROUNDS=$r timeout -k 10 120 ./syrk_ab 8 0 > ../../gpurun_out/syrk_r$r.log 2>&1) || { tail gpurun_out/syrk_r$r.log; exit 1; }
  echo "rounds=$r $(cat gpurun_out/syrk_r$r.log)"
done
for r in 1 2 3; do
  KFAC_SYRK_ROUNDS=$r timeout -k 10 200 python bench.py --no-cpu-baseline --no-e2e --no-serial > gpurun_out/br$r.log 2>&1 || { tail -5 gpurun_out/br$r.log; exit 1; }
  python -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; b=d['breakdown']; print(sys.argv[1], '%.3e'%d['value'], 'ms/step %.3f'%d['ms_per_step'], 'tiles %.3f inv %.3f'%(b['factor_tiles_ms_per_step'], b['invert_ms_per_step']), 'frac %.3f'%r['frac'])" gpurun_out/br$r.log
done
