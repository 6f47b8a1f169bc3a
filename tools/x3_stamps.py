"""Timeline of one kfac_factor_tiles_x3 launch of the MLP pass, per workgroup (the
diagnostic build: bash tools/build_ab.sh stamps -DKFAC_X3_STAMPS=1).

    BNN_KFAC_AMD_LIB=ab_libs/stamps/libkfac_hip.so python tools/x3_stamps.py [mlp]

Prints, over the last launch of a pass: start / loop / end spread (realtime, 100 MHz),
the effective shader clock in the loop (s_memtime cycles / realtime), per block-mask
loop time per stage, and the end-time distribution (the tail).
"""
import ctypes
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bnn_kfac_amd import _native as N  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "mlp"
    dev = torch.device("cuda:0")
    batch, images = bench.SHAPES[(cfg, 1)]
    net = bench.build_model(cfg, dev)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    recs = bench.synthetic_records(bench.CONFIGS[cfg], images, dev, seed=1234)
    kfac = KFAC(net)
    kfac.launch_first = 16
    starts = list(range(0, images, batch))

    def one_pass():
        kfac.reset()
        for i in starts:
            for layer, (a, g) in zip(layers, recs):
                kfac.record[layer] = [a[i:i + batch], g[i:i + batch]]
            kfac.update(batch_size=min(batch, images - i))
        kfac.flush()

    for _ in range(3):
        one_pass()
    torch.cuda.synchronize()
    # the first launch of a pass (14 full batches): run a pass up to it
    kfac.reset()
    for i in starts[:-1]:
        for layer, (a, g) in zip(layers, recs):
            kfac.record[layer] = [a[i:i + batch], g[i:i + batch]]
        kfac.update(batch_size=batch)
    kfac._launch_queue()
    torch.cuda.synchronize()
    buf = np.zeros(8192 * 8, dtype=np.uint64)
    fn = N._lib.kfac_debug_x3_stamps
    fn.argtypes = [ctypes.c_void_p, ctypes.c_size_t]
    assert fn(buf.ctypes.data, buf.nbytes) == 0
    s = buf.reshape(8192, 8).astype(np.int64)
    used = s[:, 3] > 0
    s = s[used]
    t0 = s[:, 0].min()
    rt = (s[:, :4] - t0) / 100.0  # us (100 MHz)
    full = (s[:, 7] >> 16) > 0  # x3 tasks (narrow tasks leave words 1, 2, 4, 5, 7 stale)
    mask = (s[:, 7] >> 8) & 0xFF
    ns = s[:, 7] >> 16
    loop_us = rt[:, 2] - rt[:, 1]
    cyc = (s[:, 5] - s[:, 4]).astype(np.float64)
    out = {"blocks": int(used.sum()), "launch_span_us": float(rt[:, 3].max()),
           "start_us": np.percentile(rt[:, 0], [0, 50, 100]).round(2).tolist(),
           "loop_start_us": np.percentile(rt[full, 1], [0, 50, 100]).round(2).tolist(),
           "end_us_p0_p10_p50_p90_p100": np.percentile(rt[:, 3], [0, 10, 50, 90, 100]).round(2).tolist(),
           "clock_ghz_in_loop": float(np.median(cyc[full] / (loop_us[full] * 1e3)))}
    for m in sorted(set(mask[full].tolist())):
        sel = full & (mask == m)
        per = loop_us[sel] / np.maximum(ns[sel], 1)
        out[f"mask{m}"] = {"tasks": int(sel.sum()), "stages": np.percentile(ns[sel], [0, 100]).tolist(),
                           "loop_us_p50_p100": np.percentile(loop_us[sel], [50, 100]).round(2).tolist(),
                           "ns_per_stage_p50": round(float(np.median(per)) * 1e3, 1),
                           "epilogue_us_p50": round(float(np.median(rt[sel, 3] - rt[sel, 2])), 2),
                           "prologue_us_p50": round(float(np.median(rt[sel, 1] - rt[sel, 0])), 2)}
    narrow = ~full
    if narrow.any():
        out["narrow_end_us_p50_p100"] = np.percentile(rt[narrow, 3], [50, 100]).round(2).tolist()
    for m in sorted(set(mask[full].tolist())):
        sel = full & (mask == m)
        out[f"mask{m}"]["end_us_p50_p100"] = np.percentile(rt[sel, 3], [50, 100]).round(2).tolist()
    # per-SIMD load: HW_ID bits (gfx9): wave 3:0, simd 5:4, cu 11:8, sh 12, se 15:13
    hw = s[:, 6]
    simd = (s[:, 7] & 0xFF) * 10000 + ((hw >> 13) & 7) * 1000 + ((hw >> 12) & 1) * 100 + ((hw >> 8) & 15) * 10 + ((hw >> 4) & 3)
    cu = simd // 10
    _, cnt = np.unique(cu, return_counts=True)
    out["workgroups_per_cu"] = np.bincount(cnt).tolist()
    print(json.dumps(out, indent=1), flush=True)


if __name__ == "__main__":
    main()
