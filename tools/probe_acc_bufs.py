"""A/B probe: the pipelined MLP loop with 2 or 3 accumulator buffers taken in turn by
the passes whose reduce runs on the inversion's side stream (KFAC._acc_bufs).  With 2,
the pass k+1 launch waits (a stream wait packet) for the side reduce of pass k-1 unless
the host already sees it complete; with 3 the buffer it takes was read three passes ago.
Alternates the settings in one process, `reps` times each; prints ms/step.

    python tools/probe_acc_bufs.py [steps] [reps]
"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from bnn_kfac_amd import _native as N  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    specs = bench.CONFIGS["mlp"]
    batch, images = bench.SHAPES[("mlp", 1)]
    net = bench.build_model("mlp", dev)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(specs, images, dev, seed=1234)
    starts = list(range(0, images, batch))
    views = [[(layer, [a[i:i + batch], g[i:i + batch]]) for layer, (a, g) in zip(layers, recs)]
             for i in starts]
    sizes = [min(batch, images - i) for i in starts]
    kfac = KFAC(net)
    kfac.eager_verdict = False
    kfac.launch_first = 16
    waits = {"n": 0}
    real_wait = N.RawEvent.wait_on

    def counting_wait(self, stream):
        waits["n"] += 1
        return real_wait(self, stream)

    N.RawEvent.wait_on = counting_wait

    def one_pass():
        kfac.reset()
        for batch_views, size in zip(views, sizes):
            for layer, rec in batch_views:
                kfac.record[layer] = rec
            kfac.update(batch_size=size)
        kfac.invert(*bench.DAMPING)

    out = {2: [], 3: []}
    for rep in range(reps):
        for nbuf in (2, 3):
            kfac.inv_state
            torch.cuda.synchronize(dev)
            kfac._acc_bufs = [None] * nbuf
            kfac._acc_par = 0
            kfac._acc_reads = {}
            for _ in range(10):
                one_pass()
            kfac.inv_state
            torch.cuda.synchronize(dev)
            waits["n"] = 0
            t0 = time.perf_counter()
            for _ in range(steps):
                one_pass()
            kfac.inv_state
            torch.cuda.synchronize(dev)
            ms = 1e3 * (time.perf_counter() - t0) / steps
            out[nbuf].append(round(ms, 4))
            print(f"rep {rep} nbuf={nbuf}: {ms:.4f} ms/step, {waits['n'] / steps:.2f} event waits per step",
                  flush=True)
    print(json.dumps({"steps": steps, "nbuf2_ms": out[2], "nbuf3_ms": out[3]}), flush=True)


if __name__ == "__main__":
    main()
