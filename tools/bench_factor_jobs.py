"""Time kfac_factor_update per factor job (one job per call) for a bench config, to
see which operand layouts/shapes dominate a grouped update.  GPU only."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bnn_kfac_amd import _native as N  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "lenet"
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    dev = torch.device("cuda:0")
    specs = bench.CONFIGS[cfg]
    net = bench.build_model(cfg, dev)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    recs = bench.synthetic_records(specs, batch, dev, seed=0)
    res = {}
    for li, (layer, spec, (a, g)) in enumerate(zip(layers, specs, recs)):
        opA, opG, _nA, _nG, _keep = KFAC._operands(layer, a, g)
        for name, op in (("A", opA), ("G", opG)):
            n = op.cols + (1 if op.has_ones else 0)
            F = torch.zeros(n, n, device=dev)
            job = [N.factor_job(op, F, 1.0 / op.rows, 0.0)]
            for _ in range(3):
                N.factor_update(job, dev)
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            reps = 20
            s.record()
            for _ in range(reps):
                N.factor_update(job, dev)
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / reps * 1e3
            flops = op.rows * n * (n + 1)
            res[f"L{li}{name} n={n} rows={op.rows} layout={op.layout}"] = {
                "us": round(us, 1), "TF": round(flops / us / 1e6, 2)}
    # all jobs in one grouped call (what KFAC.update issues)
    jobs, keep = [], []
    for layer, (a, g) in zip(layers, recs):
        opA, opG, nA, nG, k = KFAC._operands(layer, a, g)
        keep.append(k)
        for op, n in ((opA, nA), (opG, nG)):
            F = torch.zeros(n, n, device=dev)
            keep.append(F)
            jobs.append(N.factor_job(op, F, 1.0 / op.rows, 0.0))
    for _ in range(3):
        N.factor_update(jobs, dev)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(10):
        N.factor_update(jobs, dev)
    e.record()
    torch.cuda.synchronize()
    res["grouped_all_jobs"] = {"us": round(s.elapsed_time(e) / 10 * 1e3, 1)}
    res["sum_of_single_jobs_us"] = round(sum(v["us"] for v in res.values() if "TF" in v), 1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
