"""Per-kernel register / spill / occupancy table from hipcc -Rpass-analysis=kernel-resource-usage
remarks:  hipcc ... -Rpass-analysis=kernel-resource-usage 2>&1 | python tools/kres.py [filter]"""
import re
import subprocess
import sys

rows, cur = [], None
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    m = re.search(r"(VGPRs|AGPRs|SGPRs|Occupancy \[waves/SIMD\]|SGPRs Spill|VGPRs Spill|LDS Size \[bytes/block\]): (\d+)", line)
    if m and cur is not None:
        cur[m.group(1).split(" [")[0]] = int(m.group(2))
flt = sys.argv[1] if len(sys.argv) > 1 else ""
names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                       text=True).stdout.splitlines()
for r, n in zip(rows, names):
    if flt in n:
        print(f"{r.get('VGPRs', 0):4d}v {r.get('AGPRs', 0):3d}a occ {r.get('Occupancy', 0)} "
              f"spill v{r.get('VGPRs Spill', 0)} s{r.get('SGPRs Spill', 0)} lds {r.get('LDS Size', 0):6d}  {n[:110]}")
