"""Host and GPU timeline of the bench's pipelined MLP step (bench.py one_pass: reset,
15 updates, invert), without a profiler: host perf_counter marks and torch.cuda
events on the caller's stream at the same points, plus the library's per-kernel HIP
events.  Prints per-step means: when the host reaches each mark, when the GPU
main stream reaches it, and how long the main stream sat idle.

    python tools/step_timeline.py [steps]
"""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bnn_kfac_amd import _native as N  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    dev = torch.device("cuda:0")
    batch, images = bench.SHAPES[("mlp", 1)]
    net = bench.build_model("mlp", dev)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(bench.CONFIGS["mlp"], images, dev, seed=1234)
    kfac = KFAC(net)
    kfac.launch_first = 16
    kfac.eager_verdict = False
    starts = list(range(0, images, batch))
    views = [[(layer, [a[i:i + batch], g[i:i + batch]]) for layer, (a, g) in zip(layers, recs)] for i in starts]
    sizes = [min(batch, images - i) for i in starts]
    marks = ["step", "updates_done", "flushed", "inverted"]

    def one_pass(rec):
        rec["step"] = (time.perf_counter(), torch.cuda.Event(enable_timing=True))
        rec["step"][1].record()
        kfac.reset()
        for bv, size in zip(views, sizes):
            for layer, r in bv:
                kfac.record[layer] = r
            kfac.update(batch_size=size)
        rec["updates_done"] = (time.perf_counter(), torch.cuda.Event(enable_timing=True))
        rec["updates_done"][1].record()
        kfac.flush()
        rec["flushed"] = (time.perf_counter(), torch.cuda.Event(enable_timing=True))
        rec["flushed"][1].record()
        kfac.invert(*bench.DAMPING)
        rec["inverted"] = (time.perf_counter(), torch.cuda.Event(enable_timing=True))
        rec["inverted"][1].record()

    # GPU intervals of the main stream's launches: events around every factor_update /
    # factor_flush call (recorded on the caller's stream, where the launches go)
    spans = []
    live = {"on": False}

    def wrap(fn, name):
        def inner(*a, **k):
            if not live["on"]:
                return fn(*a, **k)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            r = fn(*a, **k)
            e1.record()
            spans.append((name, e0, e1))
            return r
        return inner

    N.factor_update = wrap(N.factor_update, "update")
    N.factor_flush = wrap(N.factor_flush, "reduce")
    for _ in range(5):
        one_pass({})
    torch.cuda.synchronize()
    recs_ = [{} for _ in range(steps)]
    live["on"] = True
    t0 = time.perf_counter()
    for r in recs_:
        one_pass(r)
    kfac.inv_state
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / steps
    h0, g0 = recs_[0]["step"]
    host = {m: [] for m in marks}
    gpu = {m: [] for m in marks}
    for r in recs_:
        for m in marks:
            host[m].append((r[m][0] - h0) * 1e3)
            gpu[m].append(g0.elapsed_time(r[m][1]))
    out = {"ms_per_step": round(wall * 1e3, 4)}
    # per mark: host time into the step, and (GPU - host) time of the mark on a common
    # origin (step 0's start; the origin's own lag is unknown, so only differences
    # between marks mean something: where (GPU - host) is smallest the stream had
    # drained and waited for the host)
    for m in marks:
        dh = np.array(host[m]) - np.array(host["step"])
        lag = np.array(gpu[m]) - np.array(host[m])
        out[m] = {"host_ms_into_step": round(float(np.median(dh)), 4), "gpu_minus_host_ms": round(float(np.median(lag)), 4)}
    # main-stream busy / idle from the launch spans
    ts = sorted((g0.elapsed_time(a), g0.elapsed_time(b), n) for n, a, b in spans)
    busy = {}
    idle = []
    for i, (a, b, n) in enumerate(ts):
        busy.setdefault(n, []).append(b - a)
        if i:
            idle.append(a - ts[i - 1][1])
    out["launch_ms"] = {n: [round(float(np.median(v)), 4), len(v) // steps] for n, v in busy.items()}
    out["update_spans_ms_first_two"] = [round(b - a, 4) for a, b, n in ts[:3]]
    out["main_idle_ms_per_step"] = round(float(np.sum(idle)) / steps, 4)
    out["main_busy_ms_per_step"] = round(float(sum(b - a for a, b, _ in ts)) / steps, 4)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
