"""Probe: how the pipelined MLP step time evolves from a cold start, the way bench.py
times it (W warmup passes, then blocks of K timed passes, each block bracketed by a
device sync as the bench's timed region is).  Per block: ms/step, the host's issue time per
step (and its median one_pass call), and the caching allocator's segment allocations
(hipMalloc calls) made inside it.

    python tools/probe_warm.py [W] [K] [blocks] [pre_s] [prof|noprof] [idle_s] [legs|legs+serial]

pre_s > 0: first keep the GPU busy with unrelated work (bf16 GEMMs) for that long, to
tell a power/clock ramp (then block 0 is already fast) from a warm-up of this code.
"""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def main():
    warm = int(sys.argv[1]) if len(sys.argv) > 1 else 5
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    blocks = int(sys.argv[3]) if len(sys.argv) > 3 else 12
    pre = float(sys.argv[4]) if len(sys.argv) > 4 else 0.0
    prof = len(sys.argv) > 5 and sys.argv[5] == "prof"  # the library's per-launch HIP events
    idle = float(sys.argv[6]) if len(sys.argv) > 6 else 0.0  # an idle pause before the second half
    from bnn_kfac_amd import _native as N
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    torch.cuda.set_stream(torch.cuda.Stream(dev))
    specs = bench.CONFIGS["mlp"]
    batch, images = bench.SHAPES[("mlp", 1)]
    net = bench.build_model("mlp", dev)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
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

    def segs():
        return torch.cuda.memory_stats(dev).get("segment.all.allocated", 0)

    # "legs": the bench's C5 / C3 legs first; "legs+serial": then 20 serial passes, as
    # bench.py orders them before the headline
    mode = sys.argv[7] if len(sys.argv) > 7 else ""
    if mode.startswith("legs"):
        bench.other_config("wide", dev, steps=10, warmup=2)
        bench.other_config("lenet", dev, steps=20, warmup=2)
        torch.cuda.empty_cache()
    if mode == "legs+serial":
        kfac.overlap_invert = False
        kfac.launch_first = 1
        for _ in range(21):
            one_pass()
            kfac.inv_state
            torch.cuda.synchronize(dev)
        kfac.overlap_invert = True
        kfac.launch_first = 16
    if pre > 0:
        x = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < pre:
            for _ in range(20):
                y = x @ x
            torch.cuda.synchronize(dev)
        del x, y
    for _ in range(warm):
        one_pass()
    kfac.inv_state
    torch.cuda.synchronize(dev)
    out = []
    for b in range(blocks):
        if idle > 0 and b == blocks // 2:
            time.sleep(idle)
            print(f"(idle {idle} s)", flush=True)
        s0 = segs()
        if prof:
            N.profile_reset()
            N.profile_enable(True)
        t0 = time.perf_counter()
        host = []
        for _ in range(steps):
            h0 = time.perf_counter()
            one_pass()
            host.append(time.perf_counter() - h0)
        t_issue = time.perf_counter() - t0
        kfac.inv_state
        torch.cuda.synchronize(dev)
        ms = 1e3 * (time.perf_counter() - t0) / steps
        kern = ""
        if prof:
            N.profile_enable(False)
            x3, nx = N.profile_read(N.PROF_FACTOR_X3)
            inv, ni = N.profile_read(N.PROF_INVERT)
            kern = f", x3 {1e3 * x3 / max(nx, 1):.1f} us/launch, invert {1e3 * inv / max(ni, 1):.1f} us"
        host.sort()
        med = 1e3 * host[len(host) // 2]
        out.append((round(ms, 4), round(1e3 * t_issue / steps, 4), round(med, 4), segs() - s0))
        print(f"block {b}: {ms:.4f} ms/step, host issue {1e3 * t_issue / steps:.4f} ms/step "
              f"(median pass call {med:.4f}), {segs() - s0} new segments{kern}", flush=True)
    print(json.dumps({"warmup": warm, "steps": steps, "pre_s": pre, "blocks": out}), flush=True)


if __name__ == "__main__":
    main()
