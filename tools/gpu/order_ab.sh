# Wide-MLP A/B of the SYRK task order (KFAC_SYRK_ORDER 1 split-major, 0 tile-major):
# bench lines + one FETCH_SIZE pass each.
set -o pipefail
mkdir -p gpurun_out/order_ab
export TMPDIR=/tmp
B="python3 bench.py --config wide --steps 3 --warmup 1 --images 16384 --no-cpu-baseline --no-e2e"
for o in 1 0 1 0; do
  KFAC_SYRK_ORDER=$o timeout -k 10 300 $B > gpurun_out/order_ab/bench_$o.log 2>&1 || exit $?
  echo "order=$o $(tail -1 gpurun_out/order_ab/bench_$o.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(round(d["value"]), d["breakdown"]["factor_tiles_ms_per_step"])')"
done
for o in 1 0; do
  KFAC_SYRK_ORDER=$o timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex kfac_factor_tiles --output-format csv -d gpurun_out/order_ab/pmc_$o -o run -- $B > gpurun_out/order_ab/pmc_$o.log 2>&1 || exit $?
  python3 -c "import csv,glob; v=[float(r['Counter_Value']) for f in glob.glob('gpurun_out/order_ab/pmc_$o/**/run_counter_collection.csv', recursive=True) for r in csv.DictReader(open(f))]; print('order=$o FETCH_SIZE KiB/launch', sum(v)/len(v))"
done
