"""Host-side cost of KFAC.update / invert on a bench setup (GPU box).

    python tools/host_overhead.py [mlp|lenet|wide]
"""
import cProfile
import io
import os
import pstats
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    config = sys.argv[1] if len(sys.argv) > 1 else "mlp"
    B, images = bench.SHAPES[(config, 1)][:2]
    specs = bench.CONFIGS[config]
    net = bench.build_model(config, dev)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    recs = bench.synthetic_records(specs, images, dev, seed=0)
    kfac = KFAC(net)
    kfac.eager_verdict = False
    starts = list(range(0, images, B))

    def one_pass():
        kfac.reset()
        for i in starts:
            for layer, (a, g) in zip(layers, recs):
                kfac.record[layer] = [a[i:i + B], g[i:i + B]]
            kfac.update(batch_size=B)
        kfac.invert(0.04, 200)

    for _ in range(3):
        one_pass()
    torch.cuda.synchronize()
    # host time per pass with the GPU never the bottleneck: measure issue time only
    reps = 20
    t0 = time.perf_counter()
    for _ in range(reps):
        one_pass()
    t_issue = (time.perf_counter() - t0) / reps
    torch.cuda.synchronize()
    t_total = (time.perf_counter() - t0) / reps
    print(f"host issue time per pass {t_issue*1e3:.3f} ms, wall per pass {t_total*1e3:.3f} ms, "
          f"per update ~{t_issue/len(starts)*1e6:.1f} us (incl. invert share)")
    # pure host cost of update(): issue many without any sync (the GPU queue absorbs them)
    torch.cuda.synchronize()
    n_up = 150
    t0 = time.perf_counter()
    for k in range(n_up):
        i = starts[k % len(starts)]
        for layer, (a, g) in zip(layers, recs):
            kfac.record[layer] = [a[i:i + B], g[i:i + B]]
        kfac.update(batch_size=B)
    t_host = (time.perf_counter() - t0) / n_up
    torch.cuda.synchronize()
    t_all = (time.perf_counter() - t0) / n_up
    print(f"update(): host {t_host*1e6:.1f} us/call (incl. record slicing), GPU-bound wall {t_all*1e6:.1f} us/call")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(5):
        one_pass()
    pr.disable()
    torch.cuda.synchronize()
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(18)
    print(s.getvalue()[:4000])


if __name__ == "__main__":
    main()
