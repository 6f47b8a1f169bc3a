# Kernel stats of the wide MLP inversion (blocked updates) under rocprofv3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/wp -o run -- python3 bench.py --config wide --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-serial > gpurun_out/wp.log 2>&1 || { tail -5 gpurun_out/wp.log; exit 1; }
python tools/kstats.py gpurun_out/wp | head -12
f=$(find gpurun_out/wp -name "*kernel_trace.csv" | head -1)
python - "$f" <<'PY'
import csv, sys, collections
rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
inv = [r for r in rows if "inv_" in r["Kernel_Name"]]
# last inversion: from the last inv_build
last = max(i for i, r in enumerate(inv) if "inv_build" in r["Kernel_Name"])
seq = inv[last:]
t0 = int(seq[0]["Start_Timestamp"]); t1 = int(seq[-1]["End_Timestamp"])
busy = collections.defaultdict(float)
for r in seq:
    busy[r["Kernel_Name"].split("(")[0]] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
print("last inversion span %.1f us, %d launches" % ((t1 - t0) / 1e3, len(seq)))
for k, v in sorted(busy.items(), key=lambda x: -x[1]): print("  %-40s %9.1f us" % (k, v))
big = sorted(seq, key=lambda r: int(r["Start_Timestamp"]) - int(r["End_Timestamp"]))[:8]
for r in big: print("  top", r["Kernel_Name"].split("(")[0], r["Grid_Size_X"], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
PY
