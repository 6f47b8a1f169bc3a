# Round 4: one launch per flush (tail tasks at the end of the main launch, per-job
# accumulator slab ranges): parity, then bench A/B of KFAC_X3_TAIL / KFAC_MERGE_LAUNCHES
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04ae
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py tests/test_gpu_boundary.py -x -q --timeout 200 --timeout-method thread > $O/tests.log 2>&1 || { tail -40 $O/tests.log; exit 1; }
echo "parity: $(tail -1 $O/tests.log)"
BNN_KFAC_AMD_LIB=ab_libs/stamps/libkfac_hip.so timeout -k 10 200 python tools/x3_stamps.py mlp > $O/stamps.json 2>&1 || { tail -20 $O/stamps.json; exit 1; }
grep -v amdgpu $O/stamps.json | python -c "import json,sys; d=json.load(sys.stdin); print(json.dumps({k: d[k] for k in d if k not in ('workgroups_per_cu',)}))"
for v in "1 1" "0 0" "1 1" "0 1" "1 0" "0 0"; do
  set -- $v
  KFAC_MERGE_LAUNCHES=$1 KFAC_X3_TAIL=$2 timeout -k 10 200 python bench.py --steps 200 --warmup 20 --no-cpu-baseline --no-e2e --no-serial > $O/bench_$1$2.log 2>&1 || { tail -20 $O/bench_$1$2.log; exit 1; }
  echo "merge $1 tail $2: $(python -c "import json;d=json.loads(open('$O/bench_$1$2.log').read().strip().splitlines()[-1]);print(round(d['value']/1e6,2), round(d['ms_per_step'],4), round(d['roofline']['achieved'],1))")"
done
