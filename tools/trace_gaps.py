"""Per-queue timeline of a rocprofv3 kernel trace (kernel_trace.csv): busy time per
kernel family, idle gaps on each queue, and how much of the main queue's idle time the
side queues were busy.  python tools/trace_gaps.py <kernel_trace.csv> [last_ms]
"""
import collections
import csv
import sys


def family(name):
    for key in ("kfac_factor_tiles_x3", "kfac_factor_reduce", "kfac_factor_flush", "inv_step", "inv_build",
                "inv_out", "inv_bulk", "inv_panel", "inv_update", "kfac_factor_syrk3", "kfac_split3",
                "kfac_factor"):
        if key in name:
            return key
    return name.split("(")[0][-40:]


def main():
    path = sys.argv[1]
    last_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 5.0
    rows = list(csv.DictReader(open(path)))
    ks = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Queue_Id"], family(r["Kernel_Name"]))
          for r in rows]
    ks.sort()
    t_end = max(e for _, e, _, _ in ks)
    t0 = t_end - last_ms * 1e6
    ks = [k for k in ks if k[0] >= t0]
    span = (t_end - ks[0][0]) / 1e3
    by_q = collections.defaultdict(list)
    for s, e, q, f in ks:
        by_q[q].append((s, e, f))
    out = {"window_us": round(span, 1)}
    for q, lst in by_q.items():
        busy = collections.Counter()
        gaps = []
        prev = None
        for s, e, f in lst:
            busy[f] += (e - s) / 1e3
            if prev is not None and s > prev:
                gaps.append((s - prev) / 1e3)
            prev = max(prev or 0, e)
        out[f"queue {q}"] = {"kernels": len(lst), "busy_us": {k: round(v, 1) for k, v in busy.most_common()},
                             "idle_us": round(sum(gaps), 1), "gaps_over_5us": sorted(round(g, 1) for g in gaps
                                                                                      if g > 5)[-12:]}
    for k, v in out.items():
        print(k, v)


if __name__ == "__main__":
    main()
