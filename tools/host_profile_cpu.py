"""Profile the HOST cost of KFAC.update (Python + ctypes job building) on the CPU:
the device calls are replaced by no-ops and the device check is lifted, so what is
timed is exactly what the caller's thread spends per update() on the GPU box.

    python tools/host_profile_cpu.py lenet [updates] [--cprofile]
"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from bnn_kfac_amd import _native as N  # noqa: E402
from bnn_kfac_amd import curvatures  # noqa: E402


def main():
    config = sys.argv[1] if len(sys.argv) > 1 else "lenet"
    nup = int(sys.argv[2]) if len(sys.argv) > 2 and sys.argv[2].isdigit() else 200
    batch = bench.SHAPES[(config, 1)][0]
    for name in ("factor_update", "factor_flush"):
        setattr(N, name, lambda *a, **k: None)
    N.factor_accum_plan = lambda jobs: [(1, 256) for _ in jobs]
    N.require_device = lambda *a, **k: None
    curvatures.N = N
    dev = torch.device("cpu")
    net = bench.build_model(config, dev)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    recs = bench.synthetic_records(bench.CONFIGS[config], batch, dev, seed=0)
    kfac = curvatures.KFAC(net)

    def run(n):
        for _ in range(n):
            for m, (a, g) in zip(layers, recs):
                kfac.record[m] = [a, g]
            kfac.update(batch)
        kfac._launch_queue() if kfac._queue else None

    run(20)
    t0 = time.perf_counter()
    run(nup)
    dt = (time.perf_counter() - t0) / nup * 1e6
    print(f"{config}: {dt:.1f} us of host time per update() (batch {batch}, {len(layers)} layers)")
    if "--cprofile" in sys.argv:
        pr = cProfile.Profile()
        pr.enable()
        run(nup)
        pr.disable()
        pstats.Stats(pr).sort_stats("cumulative").print_stats(25)


if __name__ == "__main__":
    main()
