"""Turn a profiles/collect.sh run (gpurun_out/prof_<tag>/) into the committed summaries.

    python profiles/summarize.py r01          (r01_wide etc.: other configs, same recipe)

writes
  profiles/<tag>/kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (verbatim)
  profiles/<tag>/pmc_summary.json   per-kernel mean counter value per dispatch, every pass
  profiles/factor_tiles_pmc.json    HBM bytes per kfac_factor_tiles launch (read by bench.py)

HBM bytes follow MI355X_MICROARCH.md's rocprofv3 section: FETCH_SIZE and WRITE_SIZE
come from separate passes (KiB units); on gfx950 FETCH_SIZE reports half the bytes of
a wide (16 B/lane) coalesced read, so it is doubled.  Both the SYRK panel loads
(global_load_lds_dwordx4 / global_load_dwordx4) and the slab stores are 16 B/lane or
full 128-B rows.
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FETCH_X3_SCALE = 2.0  # FETCH_SIZE -> bytes for kfac_factor_tiles_x3's loads (see fetch_calib)


def short(name):
    """'void kfac::kfac_factor_tiles_t<32, 2, 2, 1>(kfac::FactorArgs)' -> 'kfac_factor_tiles'"""
    base = name.split("(")[0].split("<")[0].replace("void ", "").replace("kfac::", "").strip()
    return base[:-2] if base.endswith("_t") else base


def main(tag):
    src = os.path.join(ROOT, "gpurun_out", f"prof_{tag}")
    dst = os.path.join(ROOT, "profiles", tag)
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    pmc = collections.defaultdict(dict)
    for f in sorted(glob.glob(os.path.join(src, "pmc_*", "run_counter_collection.csv"))):
        vals = collections.defaultdict(list)
        for r in csv.DictReader(open(f)):
            vals[(short(r["Kernel_Name"]), r["Counter_Name"])].append(float(r["Counter_Value"]))
        for (k, c), v in vals.items():
            pmc[k][c] = {"mean_per_dispatch": sum(v) / len(v), "dispatches": len(v)}
    # the kernel-trace stats of the same bench command (mean launch time per kernel)
    stats = {}
    for r in csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))):
        stats[short(r["Name"])] = {"calls": int(r["Calls"]), "avg_us": float(r["AverageNs"]) / 1e3}
    with open(os.path.join(dst, "pmc_summary.json"), "w") as f:
        json.dump(pmc, f, indent=1, sort_keys=True)
    # the dominant factor kernel of the run (most trace time): the fp32-MFMA SYRK, the
    # split-pass bf16x3 SYRK (wide) or the register-split one (MNIST MLP)
    cands = [k for k in ("kfac_factor_tiles", "kfac_factor_syrk3", "kfac_factor_tiles_x3")
             if "FETCH_SIZE" in pmc.get(k, {}) and k in stats]
    kname = max(cands, key=lambda k: stats[k]["calls"] * stats[k]["avg_us"]) if cands else "kfac_factor_tiles"
    t = pmc.get(kname, {})
    if "FETCH_SIZE" in t and "WRITE_SIZE" in t:
        # FETCH_SIZE scale: x2 for 16 B/lane reads (MI355X_MICROARCH.md); the x3 kernel's
        # 4 B/lane buffer loads are calibrated by tools/fetch_calib.py (FETCH_X3_SCALE)
        # (round 5: kfac_factor_syrk3 splits in the workgroup and reads fp32 rows by the
        # same 4 B/lane buffer loads as the x3 kernel)
        scale = FETCH_X3_SCALE if kname in ("kfac_factor_tiles_x3", "kfac_factor_syrk3") else 2.0
        fetch = t["FETCH_SIZE"]["mean_per_dispatch"] * 1024 * scale
        write = t["WRITE_SIZE"]["mean_per_dispatch"] * 1024
        note = (f"FETCH_SIZE x{scale:g} (gfx950 read-width correction) + WRITE_SIZE, KiB->bytes, "
                "mean over the bench's launches (15 updates per pass, last batch short)")
        if kname == "kfac_factor_syrk3":
            note += ("; kfac_factor_syrk3 (round 5: split in the workgroup, no split pass) reads "
                     "fp32 operand rows by buffer_load_dword (4 B/lane), scale as for the x3 kernel")
        if kname == "kfac_factor_tiles_x3":
            note += ("; kfac_factor_tiles_x3 reads fp32 operand rows by buffer_load_dword "
                     "(4 B/lane, 128 B per half-wave): scale calibrated on a 512 MB operand "
                     "read once (profiles/r03_x3/fetch_calib.txt)")
        out = {"kernel": kname, "tag": tag, "fetch_bytes_per_launch": fetch,
               "write_bytes_per_launch": write, "hbm_bytes_per_launch": fetch + write,
               "rocprof_trace": stats.get(kname), "note": note}
        with open(os.path.join(dst, "factor_tiles_hbm.json"), "w") as f:
            json.dump(out, f, indent=1)
        # the files bench.py reads: factor_tiles_pmc.json for the headline (MLP) profile,
        # factor_tiles_pmc_<config>.json for r02_<config> etc.
        name = "factor_tiles_pmc.json" if "_" not in tag else f"factor_tiles_pmc_{tag.split('_', 1)[1]}.json"
        with open(os.path.join(ROOT, "profiles", name), "w") as f:
            json.dump(out, f, indent=1)
        print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "r01")
