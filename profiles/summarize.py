"""Turn a profiles/collect.sh run (gpurun_out/prof_<tag>/) into the committed summaries.

    python profiles/summarize.py <tag> <config>      (config: mlp | lenet | wide)

writes
  profiles/<tag>/kernel_stats.csv    rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>/pmc_summary.json    per kernel family: mean counter value per dispatch,
                                     every --pmc pass
  profiles/pmc_<config>.json         per factor kernel family: HBM bytes per launch and
                                     the trace's calls / mean launch time (bench.py reads
                                     it for the roofline's `traffic`)

A kernel FAMILY is the kernel's name without template arguments (and without the _t
of the fp32 template kfac_factor_tiles_t): every instance of kfac_factor_conv<...>
counts as one family, as the library's profile slot KFAC_PROF_FACTOR_CONV times them.
The trace's figures per family are summed over instances (calls, total ns), so the
family's mean launch time compares with the bench's `avg_launch_us` directly.

HBM bytes follow MI355X_MICROARCH.md's rocprofv3 section: FETCH_SIZE and WRITE_SIZE
come from separate passes (KiB units); on gfx950 FETCH_SIZE reports half the bytes of
a wide coalesced read, so it is doubled (the x3 / syrk3 kernels' 4 B/lane buffer loads:
the same x2, calibrated on a 512 MB operand read once, profiles/r03_x3/fetch_calib.txt).
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FETCH_SCALE = 2.0
FACTOR_FAMILIES = ("kfac_factor_tiles", "kfac_factor_tiles_x3", "kfac_factor_syrk3", "kfac_factor_conv",
                   "kfac_factor_conv_x3", "kfac_factor_conv_x3s", "kfac_factor_conv_x3f", "kfac_factor_channel_small",
                   "kfac_factor_channel_x3",
                   "kfac_factor_reduce")


def family(name):
    """'void kfac::kfac_factor_conv<2, 8, true, 2, false>(kfac::FactorArgs, kfac::ConvGeom)'
    -> 'kfac_factor_conv'; 'kfac::t32::inv_step(...)' -> 't32::inv_step'."""
    base = name.split("(")[0].split("<")[0].replace("void ", "").replace("kfac::", "").strip()
    return base[:-2] if base.endswith("_t") else base


def main(tag, config):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    pmc = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(src, "pmc_*", "run_counter_collection.csv"))):
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            vals[(family(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in vals.items():
            pmc[k][c] = {"mean_per_dispatch": sum(v) / len(v), "dispatches": len(v)}
    # the kernel-trace stats of the same bench command, summed over each family's instances
    calls, total_ns = collections.Counter(), collections.Counter()
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        calls[family(r["Name"])] += int(r["Calls"])
        total_ns[family(r["Name"])] += float(r["TotalDurationNs"])
    stats = {k: {"calls": calls[k], "avg_us": total_ns[k] / calls[k] / 1e3, "total_ms": total_ns[k] / 1e6}
             for k in calls}
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump({"trace": stats, "pmc": pmc}, f, indent=1, sort_keys=True)
    kernels = {}
    for k in FACTOR_FAMILIES:
        t = pmc.get(k, {})
        if "FETCH_SIZE" not in t or "WRITE_SIZE" not in t:
            continue
        fetch = t["FETCH_SIZE"]["mean_per_dispatch"] * 1024 * FETCH_SCALE
        write = t["WRITE_SIZE"]["mean_per_dispatch"] * 1024
        kernels[k] = {"fetch_bytes_per_launch": fetch, "write_bytes_per_launch": write,
                      "hbm_bytes_per_launch": fetch + write, "fetch_scale": FETCH_SCALE,
                      "pmc_dispatches": t["FETCH_SIZE"]["dispatches"], "rocprof_trace": stats.get(k)}
    out = {"tag": tag, "config": config, "kernels": kernels,
           "note": "per kernel family: FETCH_SIZE x2 (gfx950 read-width correction) + WRITE_SIZE, KiB -> "
                   "bytes, mean per dispatch over the bench run's launches (separate --pmc passes); "
                   "rocprof_trace = the same command's kernel trace, summed over the family's instances"}
    with open(os.path.join(ROOT, "profiles", f"pmc_{config}.json"), "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "mlp")
