"""Kernel timeline of the last bench steps from a rocprofv3 --kernel-trace CSV:

    python tools/timeline.py <run_kernel_trace.csv> [kernels-to-show]

Prints each kfac / inversion kernel with its stream (queue), start relative to
the first shown kernel, duration, and the busy union per stream (so the overlap of
the inversion side stream with the data pass is visible)."""
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
n = int(sys.argv[2]) if len(sys.argv) > 2 else 120
kf = [r for r in rows if "kfac" in r["Kernel_Name"] or "inv_" in r["Kernel_Name"] or "tri_" in r["Kernel_Name"]]
tail = kf[-n:]
t0 = int(tail[0]["Start_Timestamp"])
qkey = "Queue_Id" if "Queue_Id" in tail[0] else ("Stream_Id" if "Stream_Id" in tail[0] else None)
busy = {}
for r in tail:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    q = r.get(qkey, "?") if qkey else "?"
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("kfac::", "")[:44]
    grid = r.get("Grid_Size_X", r.get("Grid_Size", "?"))
    print(f"q{q:>3} {name:44s} grid {grid:>8} start {(s - t0) / 1e3:9.2f} us  dur {(e - s) / 1e3:8.2f} us")
    busy.setdefault(q, []).append((s, e))
span = (int(tail[-1]["End_Timestamp"]) - t0) / 1e3
print(f"span {span:.1f} us")
for q, iv in busy.items():
    iv.sort()
    tot, cs, ce = 0, None, None
    for s, e in iv:
        if cs is None or s > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = s, e
        else:
            ce = max(ce, e)
    tot += ce - cs
    print(f"queue {q}: busy {tot / 1e3:.1f} us of {span:.1f}")
