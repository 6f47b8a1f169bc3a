"""Inter-kernel gaps of one bench pass from a rocprofv3 kernel trace CSV:
python tools/gaps.py gpurun_out/trace_gaps/.../run_kernel_trace.csv"""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
kf = [r for r in rows if "kfac" in r["Kernel_Name"] or "inv_" in r["Kernel_Name"]]
# last full pass: from the last-but-one inv_step(k=-1)... simply print the tail
tail = kf[-40:]
prev = None
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    gap = (s - prev) / 1e3 if prev else 0.0
    print(f"{r['Kernel_Name'].split('(')[0][:40]:40s} grid {r.get('Grid_Size_X', r.get('Grid_Size','?')):>8s} dur {(e-s)/1e3:8.2f} us  gap {gap:7.2f} us")
    prev = e
