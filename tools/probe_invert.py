"""Probe: GPU time of the MLP's grouped inversion alone (KFAC.invert on the caller's
stream, overlap off), median over `reps` of torch.cuda events around each call, on the
factors of one bench pass.  The library is the in-tree one unless BNN_KFAC_AMD_LIB
points elsewhere (same-box A/B of builds, one process each).

    python tools/probe_invert.py [reps] [tag] [config]   (config: mlp, or wide for C5)
"""
import json
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    tag = sys.argv[2] if len(sys.argv) > 2 else ""
    cfg = sys.argv[3] if len(sys.argv) > 3 else "mlp"
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    specs = bench.CONFIGS[cfg]
    batch, images = bench.SHAPES[(cfg, 1)]
    net = bench.build_model(cfg, dev)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(specs, images, dev, seed=1234)
    kfac = KFAC(net)
    kfac.overlap_invert = False
    for i in range(0, images, batch):
        for layer, (a, g) in zip(layers, recs):
            kfac.record[layer] = [a[i:i + batch], g[i:i + batch]]
        kfac.update(batch_size=min(batch, images - i))
    kfac.invert(*bench.DAMPING)
    torch.cuda.synchronize(dev)
    ts = []
    for _ in range(reps):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        kfac.invert(*bench.DAMPING)
        e1.record()
        e1.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    print(json.dumps({"tag": tag, "reps": reps, "median_ms": round(ts[len(ts) // 2], 4),
                      "p10_ms": round(ts[len(ts) // 10], 4), "p90_ms": round(ts[9 * len(ts) // 10], 4)}),
          flush=True)


if __name__ == "__main__":
    main()
