"""A/B probe: the pipelined bench loop with the pass's deferred reduce on the
inversion's side stream (KFAC.reduce_on_side, default) or on the caller's stream.
Alternates the two settings in one process, `reps` times each, and prints ms/step.

    python tools/probe_side_reduce.py [config] [steps] [reps]
"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def main():
    config = sys.argv[1] if len(sys.argv) > 1 else "mlp"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 200
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    specs = bench.CONFIGS[config]
    batch, images = bench.SHAPES[(config, 1)]
    net = bench.build_model(config, dev)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    recs = bench.synthetic_records(specs, images, dev, seed=1234)
    starts = list(range(0, images, batch))
    views = [[(layer, [a[i:i + batch], g[i:i + batch]]) for layer, (a, g) in zip(layers, recs)]
             for i in starts]
    sizes = [min(batch, images - i) for i in starts]
    kfac = KFAC(net)
    kfac.eager_verdict = False
    kfac.launch_first = 16

    def one_pass():
        kfac.reset()
        for batch_views, size in zip(views, sizes):
            for layer, rec in batch_views:
                kfac.record[layer] = rec
            kfac.update(batch_size=size)
        kfac.invert(*bench.DAMPING)

    out = {True: [], False: []}
    for rep in range(reps):
        for side in (True, False):
            kfac.reduce_on_side = side
            for _ in range(10):
                one_pass()
            kfac.inv_state
            torch.cuda.synchronize(dev)
            t0 = time.perf_counter()
            for _ in range(steps):
                one_pass()
            kfac.inv_state
            torch.cuda.synchronize(dev)
            ms = 1e3 * (time.perf_counter() - t0) / steps
            out[side].append(round(ms, 4))
            print(f"rep {rep} reduce_on_side={side}: {ms:.4f} ms/step", flush=True)
    print(json.dumps({"config": config, "steps": steps,
                      "side_ms": out[True], "main_ms": out[False]}), flush=True)


if __name__ == "__main__":
    main()
