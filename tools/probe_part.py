"""KFAC's built-in CU partition (partition_cus) on the bench loop: wall per pass and
how many accumulation cycles ran on the data stream (GPU box)."""
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

    def measure(label, overlap, part, sync_after_update=False):
        kfac = KFAC(net)
        kfac.overlap_invert = overlap
        kfac.partition_cus = part
        stats = {"busy": 0, "cycles": 0}
        orig = kfac._cycle_setup

        def wrapped(device):
            orig(device)
            stats["cycles"] += 1
            stats["busy"] += kfac._cycle_stream is not None
        kfac._cycle_setup = wrapped

        tm = {"upd": 0.0, "inv": 0.0, "chk": 0.0}

        def one_pass():
            kfac.reset()
            t0 = time.perf_counter()
            for i in starts:
                for layer, (a, g) in zip(layers, recs):
                    kfac.record[layer] = [a[i:i + 4096], g[i:i + 4096]]
                kfac.update(batch_size=4096)
            t1 = time.perf_counter()
            kfac.flush()
            _ = kfac.state
            t2 = time.perf_counter()
            kfac._check_inverse()
            t3 = time.perf_counter()
            kfac.invert(0.04, 200)
            t4 = time.perf_counter()
            tm["upd"] += t1 - t0
            tm["chk"] += t3 - t2
            tm["inv"] += t4 - t3 + t2 - t1

        for _ in range(3):
            one_pass()
        torch.cuda.synchronize()
        stats.update(busy=0, cycles=0)
        tm.update(upd=0.0, inv=0.0, chk=0.0)
        reps = 30
        t0 = time.perf_counter()
        for _ in range(reps):
            one_pass()
        host = (time.perf_counter() - t0) / reps
        torch.cuda.synchronize()
        wall = (time.perf_counter() - t0) / reps
        print(f"{label:30s} wall {wall*1e3:.3f} ms/pass ({60000/wall/1e6:.1f} M img/s) host {host*1e3:.3f} ms, "
              f"cycles on data stream {stats['busy']}/{stats['cycles']}; host ms/pass update "
              f"{tm['upd']/reps*1e3:.3f} settle {tm['chk']/reps*1e3:.3f} flush+invert {tm['inv']/reps*1e3:.3f}",
              flush=True)

    measure("serial", False, 0)
    measure("overlap, no partition", True, 0)
    measure("overlap, partition 32", True, 32)
    os.environ["KFAC_INV_TILE"] = "64"
    measure("64-tiles serial", False, 0)
    measure("64-tiles overlap", True, 0)
    os.environ.pop("KFAC_INV_TILE")
    measure("32-tiles overlap again", True, 0)


if __name__ == "__main__":
    main()
