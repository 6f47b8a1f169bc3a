# Round 5: vectorised Y clear (inversion) -- inversion tests + alone time; the serial
# figure's first launch size (bench --launch-first sets both loops; the serial figure is
# read), 2 reps
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05av
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_invert.py tests/test_gpu_invert_graph.py tests/test_gpu_golden_r02.py tests/test_gpu_c2.py tests/test_gpu_wide.py -m gpu -x -q --timeout 120 --timeout-method thread > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for r in 1 2; do timeout -k 10 120 python3 tools/probe_invert.py 300 new >> $O/invert.log 2>&1 || { tail -5 $O/invert.log; exit 1; }; done
grep median $O/invert.log
for r in 1 2; do
for lf in 1 4 8 16; do
timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --no-cpu-baseline --no-e2e --no-other-configs --launch-first $lf > $O/lf${lf}_$r.log 2>&1 || { tail -20 $O/lf${lf}_$r.log; exit 1; }
python3 -c "
import json;d=json.loads(open('$O/lf${lf}_$r.log').read().strip().splitlines()[-1])
print('lf $lf $r serial', round(d['serial_images_per_s']/1e7,3), 'pipelined', round(d['value']/1e8,4))"
done
done
run() {
  tag=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --steps 100 --warmup 20 --no-cpu-baseline --no-e2e --no-other-configs --no-serial > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1])
b=d['breakdown']
print('$tag', round(d['value']/1e8,4), round(d['ms_per_step'],4), 'x3', round(b['factor_tiles_ms_per_step'],4), 'inv', round(b['invert_ms_per_step'],4))"
}
for r in 1 2; do
run def_$r KFAC_NONE=1
run x3prio1_$r BNN_KFAC_AMD_LIB=ab_libs/x3prio1/libkfac_hip.so
run sprio0_$r KFAC_INV_STREAM_PRIO=0
done
