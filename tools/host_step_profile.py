"""Profile the HOST cost of one bench step (bench.py's pipelined one_pass: reset, the
pass's update() calls, invert()) on the CPU: every device call is a no-op and the
torch.cuda stream / event calls are stand-ins, so what is timed is the Python +
ctypes work the caller's thread does per step on the GPU box (bench's
host_issue_ms_per_step, minus the real HIP API calls' own cost).

    python tools/host_step_profile.py [mlp|lenet|wide] [steps] [--cprofile]
"""
import cProfile
import os
import pstats
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import bench  # noqa: E402
import host_double  # noqa: E402
from bnn_kfac_amd import _native as N  # noqa: E402
from bnn_kfac_amd import curvatures  # noqa: E402


class _Ev:
    def __init__(self, *a, **k):
        self.cuda_event = None

    def record(self, *a):
        pass

    def query(self):
        return True

    def synchronize(self):
        pass


class _St:
    cuda_stream = 0

    def wait_stream(self, o):
        pass

    def wait_event(self, e):
        pass


def main():
    config = sys.argv[1] if len(sys.argv) > 1 and not sys.argv[1].isdigit() else "mlp"
    steps = next((int(a) for a in sys.argv[1:] if a.isdigit()), 200)
    batch, images = bench.SHAPES[(config, 1)]
    for name in ("factor_update", "factor_flush"):
        setattr(N, name, lambda *a, **k: None)
    N.factor_accum_plan = lambda jobs: [(1, 256) for _ in jobs]
    N.require_device = lambda *a, **k: None
    N.invert = lambda jobs, device, inputs_read=None: torch.zeros(len(jobs), dtype=torch.int32)
    N.invert_pipelined = lambda jobs, device, host, *a, **k: host.zero_()
    N.RawEvent = host_double.HostRawEvent
    N.stream_handle = lambda device: 0
    st = _St()
    torch.cuda.current_stream = lambda device=None: st
    torch.cuda.Stream = lambda *a, **k: _St()
    torch.cuda.stream = host_double._NoStream
    torch.cuda.Event = _Ev
    dev = torch.device("cpu")
    net = bench.build_model(config, dev)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    recs = bench.synthetic_records(bench.CONFIGS[config], images, dev, seed=0)
    kfac = curvatures.KFAC(net)
    kfac.eager_verdict = False
    kfac.launch_first = 16
    kfac._pinned_info = lambda info: torch.empty(info.numel(), dtype=torch.int32)
    kfac._pinned_host = lambda n: torch.empty(n, dtype=torch.int32)
    for t in (torch.Tensor.record_stream,):
        pass
    torch.Tensor.record_stream = lambda self, s: None
    starts = list(range(0, images, batch))
    views = [[(layer, [a[i:i + batch], g[i:i + batch]]) for layer, (a, g) in zip(layers, recs)] for i in starts]
    sizes = [min(batch, images - i) for i in starts]
    record = kfac.record

    def one_pass():
        kfac.reset()
        for bv, size in zip(views, sizes):
            for layer, rec in bv:
                record[layer] = rec
            kfac.update(batch_size=size)
        kfac.invert(*bench.DAMPING)

    for _ in range(10):
        one_pass()
    t0 = time.perf_counter()
    for _ in range(steps):
        one_pass()
    dt = (time.perf_counter() - t0) / steps * 1e6
    print(f"{config}: {dt:.1f} us of host time per step ({len(starts)} updates + invert)")
    if "--phases" in sys.argv:
        ph = [0.0, 0.0, 0.0]
        for _ in range(steps):
            t0 = time.perf_counter()
            kfac.reset()
            t1 = time.perf_counter()
            for bv, size in zip(views, sizes):
                for layer, rec in bv:
                    record[layer] = rec
                kfac.update(batch_size=size)
            t2 = time.perf_counter()
            kfac.invert(*bench.DAMPING)
            t3 = time.perf_counter()
            ph[0] += t1 - t0
            ph[1] += t2 - t1
            ph[2] += t3 - t2
        print("reset / updates / invert: " + " / ".join(f"{1e6 * v / steps:.1f}" for v in ph) + " us per step")
    if "--cprofile" in sys.argv:
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(steps):
            one_pass()
        pr.disable()
        pstats.Stats(pr).sort_stats("tottime").print_stats(30)


if __name__ == "__main__":
    main()
