"""Probe: where a merged inversion step's time goes on its critical path.  Needs the
timing build (tools/build_ab.sh invstamps -DKFAC_INV_STAMPS=1) loaded through
BNN_KFAC_AMD_LIB: the critical workgroup of every step of the MLP's grouped inversion
(job 0 = the 785 factor) records s_memrealtime (100 MHz) at its phase boundaries.

    BNN_KFAC_AMD_LIB=ab_libs/invstamps/libkfac_hip.so python tools/probe_inv_stamps.py [reps]

Prints the mean (over steps 1 .. T-2) of each phase's duration in microseconds, the
gap from one step's exit to the next step's entry, and the whole chain.
"""
import ctypes
import json
import sys

import numpy as np
import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from bnn_kfac_amd import _native as N  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402

PHASES = ["entry", "loaded", "panel", "diag updated", "elim 0", "panel 0", "trailing 0", "elim 1",
          "panel 1", "-", "-", "-", "pivots", "stored", "emitted", "exit"]


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    specs = bench.CONFIGS["mlp"]
    batch, images = bench.SHAPES[("mlp", 1)]
    net = bench.build_model("mlp", dev)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(specs, images, dev, seed=1234)
    kfac = KFAC(net)
    kfac.overlap_invert = False
    for i in range(0, images, batch):
        for layer, (a, g) in zip(layers, recs):
            kfac.record[layer] = [a[i:i + batch], g[i:i + batch]]
        kfac.update(batch_size=min(batch, images - i))
    lib = N.lib()
    fn = lib.kfac_debug_inv_stamps
    fn.restype = ctypes.c_int
    fn.argtypes = [ctypes.c_void_p, ctypes.c_int]
    rows = []
    for _ in range(reps):
        kfac.invert(*bench.DAMPING)
        torch.cuda.synchronize(dev)
        buf = np.zeros((96, 16), dtype=np.uint64)
        assert fn(buf.ctypes.data, buf.size) == 0
        rows.append(buf.astype(np.int64))
    T = 25  # the 785 factor's 32-tiles
    st = np.stack(rows)[:, :T + 1, :]  # [rep][step + 1][phase]
    steps = st[:, 2:T, :]  # steps 1 .. T-2 (full critical path: diag task + factorisation)
    out = {}
    order = [0, 1, 2, 3, 4, 5, 6, 7, 8, 12, 13, 14, 15]
    for a, b in zip(order[:-1], order[1:]):
        d = (steps[:, :, b] - steps[:, :, a]) * 0.01  # 10 ns ticks -> us
        out[f"{PHASES[a]} -> {PHASES[b]}"] = round(float(np.median(d)), 3)
    gap = (st[:, 2:T, 0] - st[:, 1:T - 1, 15]) * 0.01
    out["exit -> next entry"] = round(float(np.median(gap)), 3)
    chain = (st[:, T, 15] - st[:, 0, 0]) * 0.01
    out["chain (step -1 entry .. step T-1 exit)"] = round(float(np.median(chain)), 2)
    per_step = (st[:, 2:T, 15] - st[:, 2:T, 0]) * 0.01
    out["critical task per step"] = round(float(np.median(per_step)), 3)
    for k, v in out.items():
        print(f"{k:45s} {v:8.3f} us", flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
