"""Time the factor pass ALONE (no inversion beside it): the bench's pipelined-loop pass
(bench.py one_pass without invert: the same queued multi-batch SYRK launches and the
deferred reduce), kernel durations from the library's own HIP events.

    python tools/syrk_alone.py [mlp|lenet|wide] [passes]
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bnn_kfac_amd import _native as N  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "mlp"
    passes = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda:0")
    batch, images = bench.SHAPES[(cfg, 1)]
    specs = bench.CONFIGS[cfg]
    net = bench.build_model(cfg, dev)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    recs = bench.synthetic_records(specs, images, dev, seed=1234)
    kfac = KFAC(net)
    kfac.launch_first = 16
    starts = list(range(0, images, batch))
    views = [[(layer, [a[i:i + batch], g[i:i + batch]]) for layer, (a, g) in zip(layers, recs)]
             for i in starts]

    def one_pass():
        kfac.reset()
        for bv, i in zip(views, starts):
            for layer, rec in bv:
                kfac.record[layer] = rec
            kfac.update(batch_size=min(batch, images - i))
        kfac.flush()

    for _ in range(3):
        one_pass()
    torch.cuda.synchronize()
    N.profile_reset()
    N.profile_enable(True)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(passes):
        one_pass()
    e1.record()
    torch.cuda.synchronize()
    N.profile_enable(False)
    out = {"config": cfg, "pass_ms": e0.elapsed_time(e1) / passes}
    for name, pid in (("tiles", N.PROF_FACTOR_TILES), ("x3", N.PROF_FACTOR_X3), ("syrk3", N.PROF_FACTOR_SYRK3),
                      ("reduce", N.PROF_FACTOR_REDUCE)):
        ms, n = N.profile_read(pid)
        if n:
            out[name + "_us_per_launch"] = 1e3 * ms / n
            out[name + "_launches_per_pass"] = n / passes
    fpi = bench.flops_per_image(specs)
    if out.get("x3_us_per_launch"):
        per_launch = fpi * images / out["x3_launches_per_pass"]
        out["x3_tflops"] = per_launch / (out["x3_us_per_launch"] * 1e-6) / 1e12
        out["x3_frac_417"] = out["x3_tflops"] / bench.SYRK3_PEAK_TFLOPS
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
