"""Host cost of the C-ABI calls one MLP bench step makes (the caller's thread only:
time.perf_counter around each call, the GPU drained every few calls so queues stay
short).  Run on the GPU box:  python tools/host_api_bench.py [reps]
"""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bnn_kfac_amd import _native as N  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def timed(fn, reps, sync_every=8):
    ts = []
    for i in range(reps):
        if i % sync_every == 0:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    torch.cuda.synchronize()
    ts.sort()
    return round(ts[len(ts) // 2] * 1e6, 2)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda:0")
    batch, images = bench.SHAPES[("mlp", 1)]
    net = bench.build_model("mlp", dev)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(bench.CONFIGS["mlp"], images, dev, seed=1234)
    kfac = KFAC(net)
    kfac.launch_first = 16
    kfac.eager_verdict = False
    starts = list(range(0, images, batch))

    def one_pass():
        kfac.reset()
        for i in starts:
            for layer, (a, g) in zip(layers, recs):
                kfac.record[layer] = [a[i:i + batch], g[i:i + batch]]
            kfac.update(batch_size=min(batch, images - i))

    for _ in range(3):
        one_pass()
        kfac.invert(*bench.DAMPING)
    torch.cuda.synchronize()
    out = {}
    out["pass_updates_only_us"] = timed(one_pass, 50, sync_every=1)
    one_pass()
    kfac.flush()
    out["invert_us"] = timed(lambda: kfac.invert(*bench.DAMPING), reps)
    # the pieces of invert(): the grouped inversion's C call with the same jobs
    st = kfac.state
    jobs, outs = [], []
    for layer in layers:
        A, G = st[layer][0], st[layer][1]
        for F in (A, G):
            o = torch.empty_like(F)
            outs.append(o)
            jobs.append(N.invert_job(F, o, 1.0, 0.2))
    main_h = N.stream_handle(dev)
    side = torch.cuda.Stream(device=dev, priority=-1)
    ev = [N.RawEvent() for _ in range(3)]
    host = torch.empty(len(jobs), dtype=torch.int32).pin_memory()
    out["invert_pipelined_us"] = timed(lambda: N.invert_pipelined(jobs, dev, host, ev[0], ev[1], ev[2], main_h,
                                                                  side.cuda_stream, side), reps)
    out["invert_plain_us"] = timed(lambda: N.invert(jobs, dev), reps)
    out["event_record_us"] = timed(lambda: ev[0].record(main_h), reps)
    out["stream_wait_us"] = timed(lambda: ev[0].wait_on(side.cuda_stream), reps)
    out["empty_like_us"] = timed(lambda: torch.empty_like(outs[0]), reps)
    x = torch.zeros(4, device=dev)
    out["torch_add_us"] = timed(lambda: x.add_(1.0), reps)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
