"""Step time of the MLP bench loop with the inversion and the data pass on disjoint CU
sets (CU-masked streams) vs the unmasked side stream vs serial (GPU box)."""
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
    ncu = N.cu_count(dev)
    print("CUs", ncu, flush=True)
    specs = bench.CONFIGS["mlp"]
    net = bench.build_model("mlp", dev)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(specs, 60000, dev, seed=0)
    starts = list(range(0, 60000, 4096))

    def measure(label, overlap, inv_cus=None, layout="balanced", invert_only=False):
        kfac = KFAC(net)
        kfac.overlap_invert = overlap
        main_stream = torch.cuda.current_stream(dev)
        if inv_cus:
            # mask bit i = XCC i % 8, local CU i // 8 (tools/microbench/cu_map.hip)
            if layout == "xcc0":  # all on XCC 0
                inv = [8 * i for i in range(inv_cus)]
            else:  # balanced: inv_cus / 8 CUs per XCC
                inv = list(range(inv_cus))
            rest = [c for c in range(ncu) if c not in set(inv)]
            main_stream = N.cu_mask_stream(dev, rest)
            kfac._inv_streams[dev.index] = N.cu_mask_stream(dev, inv)

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

        with torch.cuda.stream(main_stream):
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
        t_ms, _ = N.profile_read(N.PROF_FACTOR_TILES)
        i_ms, _ = N.profile_read(N.PROF_INVERT)
        print(f"{label:28s} wall {wall*1e3:.3f} ms/pass ({60000/wall/1e6:.1f} M img/s), "
              f"tiles {t_ms/reps:.3f} ms, invert {i_ms/reps:.3f} ms", flush=True)

    measure("serial", False)
    measure("side stream, unmasked", True)
    measure("inv on 32 CUs (k/8 per XCC)", True, 32)
    for k in (8, 16, 32):
        measure(f"inv on {k} CUs of XCC0", True, k, "xcc0")
    measure("inversion alone, 32 CUs XCC0", True, 32, "xcc0", invert_only=True)
    measure("inversion alone, 8 CUs XCC0", True, 8, "xcc0", invert_only=True)

if __name__ == "__main__":
    main()
