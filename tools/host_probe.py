"""Host time of the pieces of one pipelined bench step (GPU box): reset, each
update(), invert() -- with the GPU busy (no syncs), as in bench.py's timed loop."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    specs = bench.CONFIGS["mlp"]
    net = bench.build_model("mlp", dev)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(specs, 60000, dev, seed=0)
    kfac = KFAC(net)
    if len(sys.argv) > 1 and sys.argv[1] == "async":
        kfac.async_invert = True
    starts = list(range(0, 60000, 4096))
    T = {"reset": 0.0, "update": 0.0, "invert": 0.0, "record": 0.0}
    upd = []
    per_idx = {}

    def one_pass(meas):
        t = time.perf_counter()
        kfac.reset()
        t1 = time.perf_counter()
        for i in starts:
            for layer, (a, g) in zip(layers, recs):
                kfac.record[layer] = [a[i:i + 4096], g[i:i + 4096]]
            t2 = time.perf_counter()
            kfac.update(batch_size=min(4096, 60000 - i))
            t3 = time.perf_counter()
            if meas:
                T["record"] += t2 - t1
                T["update"] += t3 - t2
                upd.append(t3 - t2)
                per_idx.setdefault(i // 4096, []).append(t3 - t2)
            t1 = t3
        t4 = time.perf_counter()
        kfac.invert(0.04, 200)
        t5 = time.perf_counter()
        if meas:
            T["reset"] += 0  # folded into record
            T["invert"] += t5 - t4

    for _ in range(5):
        one_pass(False)
    kfac.inv_state
    torch.cuda.synchronize()
    n = 20
    t0 = time.perf_counter()
    for _ in range(n):
        one_pass(True)
    t_issue = time.perf_counter() - t0
    kfac.inv_state
    torch.cuda.synchronize()
    t_all = time.perf_counter() - t0
    print(f"per step: issue {1e3 * t_issue / n:.3f} ms, wall {1e3 * t_all / n:.3f} ms; "
          + ", ".join(f"{k} {1e3 * v / n:.3f} ms" for k, v in T.items()))
    upd.sort()
    print(f"update(): median {1e6 * upd[len(upd) // 2]:.1f} us, p90 {1e6 * upd[int(0.9 * len(upd))]:.1f} us, "
          f"max {1e6 * upd[-1]:.1f} us")
    print("update() by index in the pass (median us): " + " ".join(
        f"{k}:{1e6 * sorted(v)[len(v) // 2]:.0f}" for k, v in sorted(per_idx.items())))


if __name__ == "__main__" and (len(sys.argv) < 2 or sys.argv[1] not in ("launch", "invert", "parts")):
    main()


def probe_launch():
    """Host time inside the launching update()s: _launch_queue vs the C call."""
    import cProfile
    import pstats
    import io
    from bnn_kfac_amd import _native as N
    dev = torch.device("cuda:0")
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    specs = bench.CONFIGS["mlp"]
    net = bench.build_model("mlp", dev)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(specs, 60000, dev, seed=0)
    kfac = KFAC(net)
    starts = list(range(0, 60000, 4096))
    tc = []
    orig = N.lib().kfac_factor_update

    def timed(*a):
        t = time.perf_counter()
        r = orig(*a)
        tc.append(time.perf_counter() - t)
        return r
    N.lib().kfac_factor_update = timed

    def one_pass():
        kfac.reset()
        for i in starts:
            for layer, (a, g) in zip(layers, recs):
                kfac.record[layer] = [a[i:i + 4096], g[i:i + 4096]]
            kfac.update(batch_size=min(4096, 60000 - i))
        kfac.invert(0.04, 200)
    for _ in range(5):
        one_pass()
    tc.clear()
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(10):
        one_pass()
    pr.disable()
    torch.cuda.synchronize()
    tc.sort()
    print(f"kfac_factor_update C call: n {len(tc)}, median {1e6 * tc[len(tc) // 2]:.1f} us, max {1e6 * tc[-1]:.1f} us")
    s = io.StringIO()
    pstats.Stats(pr, stream=s).sort_stats("cumulative").print_stats(25)
    print(s.getvalue()[:5000])


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "launch":
    probe_launch()


def probe_invert():
    """cProfile of invert() in the pipelined loop (GPU busy, no syncs)."""
    import cProfile
    import pstats
    dev = torch.device("cuda:0")
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    specs = bench.CONFIGS["mlp"]
    net = bench.build_model("mlp", dev)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(specs, 60000, dev, seed=0)
    kfac = KFAC(net)
    starts = list(range(0, 60000, 4096))
    pr = cProfile.Profile()

    def one_pass(meas):
        kfac.reset()
        for i in starts:
            for layer, (a, g) in zip(layers, recs):
                kfac.record[layer] = [a[i:i + 4096], g[i:i + 4096]]
            kfac.update(batch_size=min(4096, 60000 - i))
        if meas:
            pr.enable()
        kfac.invert(0.04, 200)
        if meas:
            pr.disable()

    for _ in range(5):
        one_pass(False)
    for _ in range(20):
        one_pass(True)
    kfac.inv_state
    torch.cuda.synchronize()
    pstats.Stats(pr).sort_stats("tottime").print_stats(18)


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "invert":
    probe_invert()


def probe_invert_parts():
    """Wall time of invert()'s parts (pipelined loop): each wrapped call's total."""
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd import curvatures as CV
    dev = torch.device("cuda:0")
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    specs = bench.CONFIGS["mlp"]
    net = bench.build_model("mlp", dev)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(specs, 60000, dev, seed=0)
    kfac = KFAC(net)
    starts = list(range(0, 60000, 4096))
    acc = {}
    on = [False]

    def wrap(obj, name):
        f = getattr(obj, name)

        def g(*a, **k):
            t = time.perf_counter()
            try:
                return f(*a, **k)
            finally:
                if on[0]:
                    acc[name] = acc.get(name, 0.0) + time.perf_counter() - t
        setattr(obj, name, g)

    for nm in ("invert_prepare", "invert_phase", "factor_flush", "invert_job"):
        wrap(N, nm)
    for nm in ("_defer_verdict", "_damping", "_side_stream", "_release", "_invert_async", "flush"):
        wrap(kfac, nm)
    tot = [0.0]

    def one_pass(meas):
        kfac.reset()
        for i in starts:
            for layer, (a, g) in zip(layers, recs):
                kfac.record[layer] = [a[i:i + 4096], g[i:i + 4096]]
            kfac.update(batch_size=min(4096, 60000 - i))
        on[0] = meas
        t = time.perf_counter()
        kfac.invert(0.04, 200)
        if meas:
            tot[0] += time.perf_counter() - t
        on[0] = False

    for _ in range(5):
        one_pass(False)
    n = 20
    for _ in range(n):
        one_pass(True)
    kfac.inv_state
    torch.cuda.synchronize()
    print(f"invert(): {1e6 * tot[0] / n:.1f} us per call; " +
          ", ".join(f"{k} {1e6 * v / n:.1f}" for k, v in sorted(acc.items(), key=lambda kv: -kv[1])))


if __name__ == "__main__" and len(sys.argv) > 1 and sys.argv[1] == "parts":
    probe_invert_parts()
