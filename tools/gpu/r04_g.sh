# Round 4: raw-event pipelined invert host path (GPU suite, smoke, bench + host
# profile) and the x3 LDS-DMA ring A/B (parity, SYRK alone, bench, L2 hit counters)
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
DMA=ab_libs/dma/libkfac_hip.so
summ() { python -c "import json,sys;d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]);r=d['roofline'];print(sys.argv[2], round(d['value']/1e6,2),'M img/s', round(d['ms_per_step'],4),'ms', round(r['avg_launch_us'],1),'us', round(r['frac'],3), d['breakdown'].get('host_issue_ms_per_step'))" "$@"; }
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/gpu_tests.log 2>&1 || { tail -40 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
BNN_KFAC_AMD_LIB=$DMA timeout -k 10 300 python -u -m pytest tests/test_gpu_factors.py tests/test_gpu_c3.py tests/test_gpu_wide.py -x -q --timeout 200 --timeout-method thread > $O/dma_tests.log 2>&1 || { tail -40 $O/dma_tests.log; exit 1; }
echo "dma parity: $(tail -1 $O/dma_tests.log)"
timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_def.log 2>&1 || { tail -20 $O/alone_def.log; exit 1; }
BNN_KFAC_AMD_LIB=$DMA timeout -k 10 200 python tools/syrk_alone.py mlp 20 > $O/alone_dma.log 2>&1 || { tail -20 $O/alone_dma.log; exit 1; }
echo "alone def: $(tail -1 $O/alone_def.log)"
echo "alone dma: $(tail -1 $O/alone_dma.log)"
timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --host-profile $O/host_profile.txt > $O/bench_mlp.log 2>&1 || { tail -20 $O/bench_mlp.log; exit 1; }
summ $O/bench_mlp.log default
head -12 $O/host_profile.txt
BNN_KFAC_AMD_LIB=$DMA timeout -k 10 300 python bench.py --no-cpu-baseline --no-e2e --no-serial > $O/bench_dma.log 2>&1 || { tail -20 $O/bench_dma.log; exit 1; }
summ $O/bench_dma.log dma
for v in def dma; do
  L=""; [ $v = dma ] && L=$DMA
  for C in "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum"; do
    n=$(echo $C | tr ' ' '_')
    env_lib=$L; BNN_KFAC_AMD_LIB=${env_lib:-bnn_kfac_amd/libkfac_hip.so} timeout -s KILL 120 rocprofv3 --pmc $C --kernel-include-regex "kfac_factor_tiles_x3" --output-format csv -d $O/pmc_${v}_$n -o run -- python tools/syrk_alone.py mlp 5 > $O/pmc_${v}_$n.log 2>&1 || { echo "pmc $v $n rc=$?"; tail -5 $O/pmc_${v}_$n.log; exit 1; }
  done
done
python - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/r04g/pmc_*/**/*counter_collection.csv", recursive=True)):
    s = collections.defaultdict(float); n = collections.Counter()
    for r in csv.DictReader(open(f)):
        s[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
    print(f.split("/")[2], {k: round(v / max(1, n[k]) * 1, 1) for k, v in s.items()}, "per-dispatch-row")
PY
