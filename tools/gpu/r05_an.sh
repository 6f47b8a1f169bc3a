# Round 5: the headline's first blocks after the bench's own legs (C5, C3, serial), and
# the driver's command with and without the serial leg, inversion priority 0
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/r05an
mkdir -p $O
timeout -k 10 300 python3 tools/probe_warm.py 5 20 8 0 noprof 0 legs+serial > $O/warm_legs_serial.log 2>&1 || { tail -20 $O/warm_legs_serial.log; exit 1; }
timeout -k 10 300 python3 tools/probe_warm.py 5 20 8 0 noprof 0 legs > $O/warm_legs.log 2>&1 || { tail -20 $O/warm_legs.log; exit 1; }
grep block $O/warm_legs_serial.log
grep block $O/warm_legs.log
drv() {
  tag=$1; shift
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline "$@" > $O/$tag.log 2>&1 || { tail -20 $O/$tag.log; exit 1; }
  python3 -c "
import json;d=json.loads(open('$O/$tag.log').read().strip().splitlines()[-1])
o=d['other_configs']
print('$tag', round(d['value']/1e8,4), round(d['ms_per_step'],4), 'serial', d['serial_images_per_s'], 'C5', round(o['C5']['ms_per_step'],3), 'C3', round(o['C3']['ms_per_step'],3))"
}
drv drv_a
drv drv_noserial_a --no-serial
drv drv_b
drv drv_noserial_b --no-serial
