set -o pipefail
for kg in 4 2 1; do
  export BNN_KFAC_AMD_LIB=$PWD/tools/variants/lib_kg$kg.so
  timeout -k 10 600 python -m pytest tests/test_gpu_factors.py tests/test_gpu_distributed.py -x -q > gpurun_out/kg_t$kg.log 2>&1; rc=$?
  echo "KG=$kg tests rc=$rc $(tail -1 gpurun_out/kg_t$kg.log)"
  if [ $rc -gt 1 ]; then exit $rc; fi
  timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e > gpurun_out/kg_b$kg.log 2>&1; rc=$?
  if [ $rc -gt 1 ]; then exit $rc; fi
  python -c "import json; d=json.loads(open('gpurun_out/kg_b$kg.log').read().strip().splitlines()[-1]); print('KG=$kg', round(d['value']/1e6,2), 'M img/s', round(d['ms_per_step'],4), 'ms', {k: round(v,4) for k,v in d['breakdown'].items()})" || true
  timeout -k 10 300 python bench.py --config lenet --steps 3 --warmup 1 --no-cpu-baseline --no-e2e > gpurun_out/kg_l$kg.log 2>&1; rc=$?
  if [ $rc -gt 1 ]; then exit $rc; fi
  python -c "import json; d=json.loads(open('gpurun_out/kg_l$kg.log').read().strip().splitlines()[-1]); print('KG=$kg lenet', round(d['value']/1e6,3), 'M img/s', {k: round(v,4) for k,v in d['breakdown'].items()})" || true
done
