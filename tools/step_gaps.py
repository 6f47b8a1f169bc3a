"""Where the pipelined MLP step's time goes on the caller's stream (GPU clock).

Runs bench.py's C2 loop (pass of 15 updates + invert, deferred verdicts) and records
timing events on the caller's stream around every update() and invert() call.  An
event is timestamped when the GPU reaches it, so the elapsed time between two of
them is the stream's busy + idle time between the two calls:

    python tools/step_gaps.py [steps] [KFAC_SYRK3 etc. from the env]

Prints, per step, the caller-stream span of each update (launches happen on updates
1, 3, 7, 15 with launch_first = 1) and of invert(), then the mean split.
"""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    dev = torch.device("cuda:0")
    from bnn_kfac_amd.curvatures import KFAC
    specs = bench.CONFIGS["mlp"]
    net = bench.build_model("mlp", dev)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    kfac = KFAC(net)
    kfac.eager_verdict = False
    images, batch = 60000, 4096
    recs = bench.synthetic_records(specs, images, dev, seed=1234)
    starts = list(range(0, images, batch))
    marks = []

    def ev(tag):
        e = torch.cuda.Event(enable_timing=True)
        e.record()
        marks.append((tag, e, time.perf_counter()))

    def one_pass(k):
        kfac.reset()
        for u, i in enumerate(starts):
            for layer, (a, g) in zip(layers, recs):
                kfac.record[layer] = [a[i:i + batch], g[i:i + batch]]
            kfac.update(batch_size=min(batch, images - i))
            ev(f"u{u}")
        kfac.invert(*bench.DAMPING)
        ev("inv")

    for k in range(3):
        one_pass(k)
    kfac.inv_state
    torch.cuda.synchronize()
    marks.clear()
    ev("start")
    for k in range(steps):
        one_pass(k)
    kfac.inv_state
    torch.cuda.synchronize()
    # per-step spans between consecutive marks
    per = {}
    for (t0, e0, h0), (t1, e1, h1) in zip(marks, marks[1:]):
        per.setdefault(t1, []).append((e0.elapsed_time(e1), 1e3 * (h1 - h0)))
    total = marks[0][1].elapsed_time(marks[-1][1])
    print(f"{steps} steps: {total / steps:.3f} ms/step on the caller's stream "
          f"(host {1e3 * (marks[-1][2] - marks[0][2]) / steps:.3f} ms/step)")
    for tag in [f"u{u}" for u in range(len(starts))] + ["inv"]:
        v = per.get(tag, [])
        if v:
            g = sum(x[0] for x in v) / len(v)
            h = sum(x[1] for x in v) / len(v)
            print(f"  ..{tag:>4}: GPU {1e3 * g:8.1f} us   host {1e3 * h:8.1f} us")


if __name__ == "__main__":
    main()
