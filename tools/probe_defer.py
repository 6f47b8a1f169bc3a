"""Pass time vs KFAC.defer_batches on the MLP bench setup (GPU box): wall per pass
and the library's per-kernel HIP-event totals."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bnn_kfac_amd import _native as N  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    config = sys.argv[1] if len(sys.argv) > 1 else "mlp"
    specs = bench.CONFIGS[config]
    net = bench.build_model(config, dev)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    recs = bench.synthetic_records(specs, 60000, dev, seed=0)
    starts = list(range(0, 60000, 4096))
    for db, dr in ((1, False), (1, True), (2, True), (4, True), (8, True), (16, True), (64, True)):
        kfac = KFAC(net)
        kfac.defer_batches, kfac.defer_reduce = db, dr

        def one_pass():
            kfac.reset()
            for i in starts:
                for layer, (a, g) in zip(layers, recs):
                    kfac.record[layer] = [a[i:i + 4096], g[i:i + 4096]]
                kfac.update(batch_size=4096)
            kfac.invert(0.04, 200)

        for _ in range(3):
            one_pass()
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            one_pass()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        N.profile_reset()
        N.profile_enable(True)
        for _ in range(reps):
            one_pass()
        torch.cuda.synchronize()
        N.profile_enable(False)
        t_ms, t_n = N.profile_read(N.PROF_FACTOR_TILES)
        r_ms, r_n = N.profile_read(N.PROF_FACTOR_REDUCE)
        i_ms, _ = N.profile_read(N.PROF_INVERT)
        print(f"defer_batches {db:3d} defer_reduce {int(dr)}: wall {wall*1e3:.3f} ms/pass, "
              f"tiles {t_ms/reps:.3f} ms ({t_n/reps:.1f} launches, {1e3*t_ms/max(t_n,1):.1f} us each), "
              f"reduce {r_ms/reps:.3f} ms, invert {i_ms/reps:.3f} ms", flush=True)


if __name__ == "__main__":
    main()
