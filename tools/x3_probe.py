"""Time the MNIST MLP's grouped factor update (one launch of kfac_factor_tiles_x3 over
`rows` rows) with whatever library BNN_KFAC_AMD_LIB names -- the timing-probe
builds of factor.hip (KFAC_X3_PROBE 1 no DMA, 2 no split, 3 no MFMA) give the
attribution of the kernel's time.  GPU only; results of the probe builds are garbage.

    python tools/x3_probe.py [rows]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bnn_kfac_amd import _native as N  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
    dev = torch.device("cuda:0")
    specs = bench.CONFIGS["mlp"]
    net = bench.build_model("mlp", dev)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(specs, rows, dev, seed=0)
    jobs, keep = [], []
    for layer, (a, g) in zip(layers, recs):
        opA, opG, nA, nG, k = KFAC._operands(layer, a, g)
        keep.append(k)
        for op, n in ((opA, nA), (opG, nG)):
            F = torch.zeros(n, n, device=dev)
            keep.append(F)
            jobs.append(N.factor_job(op, F, 1.0 / op.rows, 0.0))
    for _ in range(5):
        N.factor_update(jobs, dev)
    torch.cuda.synchronize()
    N.profile_reset()
    N.profile_enable(True)
    for _ in range(20):
        N.factor_update(jobs, dev)
    torch.cuda.synchronize()
    N.profile_enable(False)
    for name, pid in (("tiles", N.PROF_FACTOR_TILES), ("x3", N.PROF_FACTOR_X3), ("reduce", N.PROF_FACTOR_REDUCE)):
        ms, n = N.profile_read(pid)
        if n:
            print(f"{os.path.basename(N.LIB_PATH)} rows={rows} {name}: {1e3 * ms / n:.1f} us x {n}")


if __name__ == "__main__":
    main()
