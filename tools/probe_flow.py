"""MLP bench loop (factor pass + invert) with the per-step inversion launches vs the
inv_flow persistent launch at several workgroup counts, serial and overlapped (GPU box)."""
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
    specs = bench.CONFIGS["mlp"]
    net = bench.build_model("mlp", dev)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(specs, 60000, dev, seed=0)
    starts = list(range(0, 60000, 4096))

    ncu = N.cu_count(dev)

    def measure(label, overlap, flow, wgs=32, invert_only=False, part=0):
        os.environ["KFAC_INV_FLOW"] = flow
        os.environ["KFAC_INV_FLOW_WGS"] = str(wgs)
        kfac = KFAC(net)
        kfac.overlap_invert = overlap
        main_stream = torch.cuda.current_stream(dev)
        N.set_cu_budget(0)
        if part:
            # mask bit i = XCC i % 8: CUs 0..part-1 = part/8 CUs on every XCC
            inv = list(range(part))
            main_stream = N.cu_mask_stream(dev, list(range(part, ncu)))
            kfac._inv_streams[dev.index] = N.cu_mask_stream(dev, inv)
            N.set_cu_budget(ncu - part)
        ctx = torch.cuda.stream(main_stream)
        ctx.__enter__()

        def one_pass():
            if invert_only and kfac._state:
                kfac.invert(0.04, 200)
                return
            kfac.reset()
            for i in starts:
                for layer, (a, g) in zip(layers, recs):
                    kfac.record[layer] = [a[i:i + 4096], g[i:i + 4096]]
                kfac.update(batch_size=4096)
            kfac.invert(0.04, 200)

        for _ in range(3):
            one_pass()
        torch.cuda.synchronize()
        reps = 30
        t0 = time.perf_counter()
        for _ in range(reps):
            one_pass()
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        kfac._check_inverse()
        N.profile_reset()
        N.profile_enable(True)
        for _ in range(5):
            one_pass()
        torch.cuda.synchronize()
        N.profile_enable(False)
        t_ms, _ = N.profile_read(N.PROF_FACTOR_TILES)
        i_ms, _ = N.profile_read(N.PROF_INVERT)
        ctx.__exit__(None, None, None)
        N.set_cu_budget(0)
        print(f"{label:34s} wall {wall*1e3:.3f} ms/pass ({60000/wall/1e6:.1f} M img/s), "
              f"tiles {t_ms/5:.3f} ms, invert {i_ms/5:.3f} ms", flush=True)

    measure("invert alone, per-step", False, "0", invert_only=True)
    for w in (16, 32, 64):
        measure(f"invert alone, flow {w}", False, "1", w, invert_only=True)
    measure("serial, per-step", False, "0")
    measure("serial, flow 32", False, "1", 32)
    measure("overlap, per-step", True, "0")
    for w in (16, 24, 32, 64):
        measure(f"overlap, flow {w}", True, "1", w)
    for p in (16, 32):
        measure(f"partition {p}, flow {p}", True, "1", p, part=p)
    measure("partition 32, per-step", True, "0", part=32)

if __name__ == "__main__":
    main()
