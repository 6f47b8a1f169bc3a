"""Probe: what the pipelined MLP step costs beyond its SYRK launch.  Alternates, in one
process, `reps` times each (200 steps, device sync around each block):

  full      bench.py's one_pass (reset, 15 updates, invert on the side stream)
  sidereduce reset, 15 updates, the pass's reduce on the inversion's side stream with
            invert()'s event order, no inversion
  noinv     reset, 15 updates, flush() (the pass's reduce on the caller's stream)
  launch    reset, 15 updates, the queue's launch only (x3 launches back to back)
  hostonly  reset, 15 updates with every device launch stubbed out (the host's own
            issue time of a pass without invert)

    python tools/probe_step_parts.py [steps] [reps]
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
    torch.cuda.set_stream(torch.cuda.Stream(dev))
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

    def updates():
        kfac.reset()
        for batch_views, size in zip(views, sizes):
            for layer, rec in batch_views:
                kfac.record[layer] = rec
            kfac.update(batch_size=size)

    def full():
        updates()
        kfac.invert(*bench.DAMPING)

    def noinv():
        updates()
        kfac.flush()

    def sidereduce():
        # the pass's reduce on the side stream with invert()'s event order, no inversion
        updates()
        jobs = kfac._take_reduce()
        if jobs:
            dev_ = dev
            main_h = N.stream_handle(dev_)
            side = kfac._side_stream(dev_, alternate=True)
            kfac._reduce_on_side(jobs, dev_, main_h, side.cuda_stream)

    def launch():
        updates()
        kfac._launch_queue()
        kfac._acc_flush = kfac._acc_map = None

    real_update = N.factor_update

    def hostonly():
        N.factor_update = lambda *a, **k: None
        try:
            launch()
        finally:
            N.factor_update = real_update

    modes = {"full": full, "sidereduce": sidereduce, "noinv": noinv, "launch": launch, "hostonly": hostonly}
    out = {m: [] for m in modes}
    for rep in range(reps):
        for name, fn in modes.items():
            for _ in range(10):
                fn()
            kfac.inv_state
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(steps):
                fn()
            kfac.inv_state
            torch.cuda.synchronize(dev)
            ms = 1e3 * (time.perf_counter() - t0) / steps
            out[name].append(round(ms, 4))
            print(f"rep {rep} {name}: {ms:.4f} ms/step", flush=True)
    print(json.dumps({"steps": steps, **out}), flush=True)


if __name__ == "__main__":
    main()
