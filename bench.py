#!/usr/bin/env python
"""Benchmark: images/sec for one full KFAC factor pass + factor inversion (MNIST MLP).

    python bench.py [--gpus N --steps K --warmup W] [--config mlp|lenet|wide]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

One STEP = one KFAC data pass over `--images` synthetic images per rank in batches
of `--batch` (one KFAC.update per batch, activations/gradients already resident in
HBM, records injected exactly as the reference's hooks leave them) + the packed
RCCL all-reduce (N > 1) + KFAC.invert(0.04, 200) (models/curvatures.py:325-398;
damping of classification_ll_block.py:72-73,106).  Weak scaling: every rank
processes the same per-rank workload; `value` = all ranks' images / wall time.

Also reported (same JSON line): the roofline of the dominant kernel
(kfac_factor_tiles, fp32 MFMA; HIP-event durations measured live on its stream),
the pass/invert split, an end-to-end variant (forward + Categorical label sample
+ CE backward + update + invert), and the CPU baseline: the reference's op
sequence (oracle/cpu_ref_torch.py, torch CPU fp32) on a bounded sample of the
same workload, on this host's cores.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec for full KFAC factor pass + factor inversion, MNIST MLP, 1/2/4/8 GPUs"
MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X dense fp32 MFMA (MI355X_MICROARCH.md, chip table)
DAMPING = (0.2 ** 2, 200)     # invert(std**2, N), classification_ll_block.py:72-73,106


class Layer:
    """A KFAC'd layer of a bench config: Linear (d_in, d_out) or Conv2d
    (C_in, C_out, kernel, padding, stride, H_in) with square images."""

    def __init__(self, kind, *p):
        self.kind = kind
        if kind == "linear":
            d_in, d_out = p
            self.in_shape, self.out_shape, self.L = (d_in,), (d_out,), 1
            self.nA, self.nG = d_in + 1, d_out
        else:
            C, Co, k, pad, st, H = p
            Ho = (H + 2 * pad - k) // st + 1
            self.k, self.pad, self.stride = k, pad, st
            self.in_shape, self.out_shape, self.L = (C, H, H), (Co, Ho, Ho), Ho * Ho
            self.nA, self.nG = C * k * k + 1, Co


CONFIGS = {
    "mlp": [Layer("linear", 784, 128), Layer("linear", 128, 10)],
    "wide": [Layer("linear", 784, 4096), Layer("linear", 4096, 4096), Layer("linear", 4096, 10)],
    # LeNet-5: conv1 1->6 k5 p2, pool, conv2 6->16 k5, pool, fc 400-120-84-10
    "lenet": [Layer("conv", 1, 6, 5, 2, 1, 28), Layer("conv", 6, 16, 5, 0, 1, 14),
              Layer("linear", 400, 120), Layer("linear", 120, 84), Layer("linear", 84, 10)],
}
NAMES = {"mlp": "MLP 784-128-10", "wide": "Wide MLP 784-4096-4096-10", "lenet": "LeNet-5"}


def flops_per_image(layers):
    """Algorithmic SYRK work: sum_layers L [n_A(n_A+1) + n_G(n_G+1)] (lower triangle incl.
    the bias ones column): MLP 650,402; LeNet-5 3,110,740."""
    return sum(l.L * (l.nA * (l.nA + 1) + l.nG * (l.nG + 1)) for l in layers)


def bytes_per_image(layers):
    return sum(4 * (int(np.prod(l.in_shape)) + int(np.prod(l.out_shape))) for l in layers)


def build_model(config, device):
    """Random-init model of the configured shape (default torch init, seed 0)."""
    torch.manual_seed(0)
    nn = torch.nn
    if config == "lenet":
        net = nn.Sequential(nn.Conv2d(1, 6, 5, padding=2), nn.ReLU(), nn.MaxPool2d(2),
                            nn.Conv2d(6, 16, 5), nn.ReLU(), nn.MaxPool2d(2), nn.Flatten(),
                            nn.Linear(400, 120), nn.ReLU(), nn.Linear(120, 84), nn.ReLU(),
                            nn.Linear(84, 10))
        return net.to(device)
    mods, layers = [], CONFIGS[config]
    for i, l in enumerate(layers):
        mods.append(nn.Linear(l.in_shape[0], l.out_shape[0]))
        if i + 1 < len(layers):
            mods.append(nn.ReLU())
    return nn.Sequential(*mods).to(device)


def synthetic_records(layers, images, device, seed):
    """Resident inputs U[0,1) (post-ReLU-like) and gradient records N(0,1), in the
    shapes the reference's hooks leave (curvatures.py:319-323)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    return [(torch.rand(images, *l.in_shape, device=device, generator=g),
             torch.randn(images, *l.out_shape, device=device, generator=g)) for l in layers]


def cpu_baseline(layers, images, batch, budget_s=12.0):
    """The reference's CPU op sequence (oracle/cpu_ref_torch.py) on the same workload,
    bounded to ~budget_s seconds of whole passes; returns (images/s, cores, sample)."""
    from oracle import cpu_ref_torch as C
    threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    rng = np.random.default_rng(0)
    recs = [(torch.from_numpy(rng.random((images, *l.in_shape), dtype=np.float32)),
             torch.from_numpy(rng.standard_normal((images, *l.out_shape), dtype=np.float32)))
            for l in layers]
    done, t0 = 0, time.perf_counter()
    passes = 0
    while True:
        state = {}
        for i in range(0, images, batch):
            for li, (l, (a, gr)) in enumerate(zip(layers, recs)):
                if l.kind == "linear":
                    C.linear_update(state, li, a[i:i + batch], gr[i:i + batch], True)
                else:
                    C.conv_update(state, li, a[i:i + batch], gr[i:i + batch], l.k, l.pad, l.stride, True)
        C.invert(state, *DAMPING)
        done += images
        passes += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return done / dt, threads, (f"{passes} full pass(es) of {images} synthetic images, batch {batch}, "
                                f"update+invert, torch {torch.__version__} CPU fp32, {threads} threads")


def load_traffic():
    path = os.path.join(ROOT, "profiles", "factor_tiles_pmc.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f).get("hbm_bytes_per_launch")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="mlp", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=4096, help="per-rank batch")
    ap.add_argument("--images", type=int, default=60000, help="images per rank per pass")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--partition", type=int, default=0,
                    help="CUs reserved for the overlapped inversion (KFAC.partition_cus; 0 = none)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)
    # all GPU work on one non-default stream (the legacy default stream would
    # serialise with the CU-masked streams of --partition)
    torch.cuda.set_stream(torch.cuda.Stream(device))

    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import KFAC
    from bnn_kfac_amd.distributed import DistributedKFAC

    specs = CONFIGS[args.config]
    net = build_model(args.config, device)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    kfac = DistributedKFAC(net) if world > 1 else KFAC(net)
    kfac.partition_cus = args.partition
    recs = synthetic_records(specs, args.images, device, seed=1234 + rank)
    starts = list(range(0, args.images, args.batch))

    def one_pass():
        kfac.reset()
        for i in starts:
            for layer, (a, g) in zip(layers, recs):
                kfac.record[layer] = [a[i:i + args.batch], g[i:i + args.batch]]
            kfac.update(batch_size=min(args.batch, args.images - i))
        kfac.invert(*DAMPING)

    def sync():
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()

    for _ in range(args.warmup):
        one_pass()
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_pass()
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)
    # Kernel durations: the same K steps again with the library's HIP-event timing
    # on (events recorded around each launch, on its stream).  Kept out of the timed
    # region above because the event packets add ~10 us per launch boundary.
    N.profile_reset()
    N.profile_enable(True)
    for _ in range(args.steps):
        one_pass()
    sync()
    N.profile_enable(False)
    tiles_ms, tiles_n = N.profile_read(N.PROF_FACTOR_TILES)
    red_ms, red_n = N.profile_read(N.PROF_FACTOR_REDUCE)
    inv_ms, inv_n = N.profile_read(N.PROF_INVERT)
    N.profile_reset()

    images_total = world * args.images * args.steps
    value = images_total / elapsed
    ms_per_step = 1e3 * elapsed / args.steps

    # roofline of the dominant kernel: algorithmic flops of one launch (= one
    # update of one batch) / its measured duration, averaged over the timed region
    fpi = flops_per_image(specs)
    flops_timed = fpi * args.images * args.steps
    achieved = flops_timed / (tiles_ms * 1e-3) / 1e12 if tiles_ms > 0 else None
    traffic = load_traffic() if args.config == "mlp" else None  # PMC summary is of the MLP run
    roofline = {"bound": "mfma", "achieved": achieved, "peak": MFMA_F32_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": (achieved / MFMA_F32_PEAK_TFLOPS) if achieved else None, "traffic": traffic,
                "kernel": "kfac_factor_tiles", "launches": tiles_n,
                "avg_launch_us": 1e3 * tiles_ms / max(tiles_n, 1),
                # a launch covers every queued update of the pass (multi-batch jobs):
                # per-launch figures are the step's algorithmic totals / its launches
                "flops_per_launch": fpi * args.images * args.steps / max(tiles_n, 1),
                "algorithmic_bytes_per_launch": bytes_per_image(specs) * args.images * args.steps
                                                / max(tiles_n, 1)}
    breakdown = {"factor_tiles_ms_per_step": tiles_ms / args.steps,
                 "factor_reduce_ms_per_step": red_ms / args.steps,
                 "invert_ms_per_step": inv_ms / args.steps,
                 "updates_per_step": len(starts)}

    e2e = None
    if not args.no_e2e and world == 1:
        x = torch.rand(args.images, *specs[0].in_shape, device=device)
        crit = torch.nn.CrossEntropyLoss()

        def e2e_pass():
            kfac.reset()
            for i in starts:
                logits = net(x[i:i + args.batch])
                labels = torch.distributions.Categorical(logits=logits).sample()
                loss = crit(logits, labels)
                net.zero_grad()
                loss.backward()
                kfac.update(batch_size=logits.shape[0])
            kfac.invert(*DAMPING)
        e2e_pass()
        sync()
        t1 = time.perf_counter()
        reps = max(1, args.steps // 2)
        for _ in range(reps):
            e2e_pass()
        sync()
        e2e = args.images * reps / (time.perf_counter() - t1)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        v, cores, sample = cpu_baseline(specs, args.images, args.batch)
        cpu = {"value": v, "unit": "images/s", "cores": cores, "kind": "port", "sample": sample}

    if rank == 0:
        out = {"metric": METRIC, "value": value, "unit": "images/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
               "data": "synthetic (resident U[0,1) activations, N(0,1) output-gradient records)",
               "config": {"workload": f"{NAMES[args.config]} KFAC factor pass over {args.images} "
                                      f"images/rank (batch {args.batch}/rank) + invert{DAMPING}",
                          "global_batch": args.batch * world, "images_per_rank": args.images,
                          "parallelism": f"dp{world}", "inversion_cus": args.partition or "shared"},
               "roofline": roofline, "cpu_baseline": cpu, "breakdown": breakdown,
               "e2e_images_per_s": e2e}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
