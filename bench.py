#!/usr/bin/env python
"""Benchmark: images/sec for one full KFAC factor pass + factor inversion (MNIST MLP).

    python bench.py [--gpus N --steps K --warmup W] [--config mlp|lenet|wide]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N

`--gpus N > 1` without a launcher's WORLD_SIZE: this process spawns the N rank
processes itself (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / a free
MASTER_PORT in each child's env) and never touches the GPU (spawn_ranks).

One STEP = one KFAC data pass over `--images` synthetic images per rank in batches
of `--batch` (one KFAC.update per batch, activations/gradients already resident in
HBM, records injected exactly as the reference's hooks leave them) + the packed
RCCL all-reduce of the factors' lower triangles (N > 1) + KFAC.invert(0.04, 200)
(models/curvatures.py:325-398; damping of classification_ll_block.py:72-73,106),
every inversion's pivot verdict read back inside the timed region.  Weak scaling:
every rank processes the same per-rank workload; `value` = all ranks' images / the
slowest rank's wall time.

Workloads (BASELINE.json configs): N = 1 runs C2 (MLP, batch 4096, 60,000 images);
N > 1 runs C4's per-rank shard (MLP, 8,192 rows per rank of each global batch
N x 8,192 -- 65,536 at N = 8 -- over 65,536 images per rank); `--config lenet` is
C3 (batch 1024), `--config wide` is C5.  `--strong`: SURVEY §8(e)'s strong-scaling
pass, a fixed 65,536 x 64 images in global batches of 65,536 split over the N ranks
(65,536 / N rows per rank and batch), "scaling": "strong".

`value` is the PIPELINED rate (`metric_variant`): invert() runs on a side stream and
its pivot verdict is read at the next invert() (KFAC.eager_verdict = False), so
inversion k overlaps pass k+1.  `serial_images_per_s` is the reference scripts' order
(classification_ll_block.py:93-106: a pass, then invert, its result read before the
next pass) = images / (T_pass + T_invert).

Also reported (same JSON line): the roofline of the dominant kernel
(kfac_factor_tiles, fp32 MFMA, or kfac_factor_syrk3, bf16x3 MFMA, for the wide
config's n >= 2048 factors; HIP-event durations measured live on its stream),
the pass/all-reduce/invert split, the serial rate (one pass, then invert on the
caller's stream, then the verdict read: the latency a caller who does not pipeline
passes sees), an end-to-end variant (forward + Categorical label sample + CE
backward + update + invert), and the CPU baseline: the reference's op sequence
(oracle/cpu_ref_torch.py, torch CPU fp32) on a bounded sample of the same
workload, on this host's cores (and on 1 thread).
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "images/sec for full KFAC factor pass + factor inversion, MNIST MLP, 1/2/4/8 GPUs"
MFMA_F32_PEAK_TFLOPS = 157.3  # MI355X dense fp32 MFMA (MI355X_MICROARCH.md, chip table)
# kfac_factor_syrk3 computes each fp32 product as six bf16 MFMA products (exact bf16x3
# split): its roofline is the dense bf16 MFMA peak / 6 in fp32-equivalent flops
MFMA_BF16_PEAK_TFLOPS = 2500.0
SYRK3_PEAK_TFLOPS = MFMA_BF16_PEAK_TFLOPS / 6
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
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
# (batch per rank, images per rank): C2 at N = 1, C4's shard at N > 1, C3, C5
SHAPES = {("mlp", 1): (4096, 60000), ("mlp", 2): (8192, 65536),
          ("lenet", 1): (1024, 60000), ("lenet", 2): (1024, 60000),
          ("wide", 1): (4096, 16384), ("wide", 2): (4096, 16384)}
BASELINE_CONFIG = {("mlp", 1): "C2", ("mlp", 2): "C4", ("lenet", 1): "C3", ("lenet", 2): "C3",
                   ("wide", 1): "C5", ("wide", 2): "C5"}


STRONG_IMAGES, STRONG_BATCH = 65536 * 64, 65536  # SURVEY §8(e) strong-scaling pass


def workload(config, world, strong=False):
    """(batch per rank, images per rank) of a run: weak scaling by default (SHAPES),
    or the fixed strong-scaling pass split over `world` ranks."""
    if strong:
        if config != "mlp":
            raise ValueError("--strong is the MLP pass of SURVEY §8(e)")
        return STRONG_BATCH // world, STRONG_IMAGES // world
    return SHAPES[(config, 1 if world == 1 else 2)]


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


def cpu_model():
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return None


def host_cpus():
    """What this process may run on: its CPU affinity, the cgroup CPU quota (cpu.max,
    None when unlimited) and OMP_NUM_THREADS."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = os.cpu_count() or 1
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, period = f.read().split()[:2]
            if q != "max":
                quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    omp = int(os.environ.get("OMP_NUM_THREADS", "0")) or None
    return {"affinity": affinity, "cgroup_quota_cpus": quota, "omp_num_threads": omp,
            "logical_cpus": os.cpu_count()}


def cpu_baseline(layers, images, batch, budget_s=12.0, threads=None):
    """The reference's CPU op sequence (oracle/cpu_ref_torch.py) on the same workload,
    bounded to ~budget_s seconds of batches (whole passes when they fit; else the
    batches done so far plus one inversion); returns (images/s, threads, sample)."""
    from oracle import cpu_ref_torch as C
    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    rng = np.random.default_rng(0)
    recs = [(torch.from_numpy(rng.random((images, *l.in_shape), dtype=np.float32)),
             torch.from_numpy(rng.standard_normal((images, *l.out_shape), dtype=np.float32)))
            for l in layers]
    done, passes, t0 = 0, 0, time.perf_counter()
    while True:
        state = {}
        for i in range(0, images, batch):
            for li, (l, (a, gr)) in enumerate(zip(layers, recs)):
                if l.kind == "linear":
                    C.linear_update(state, li, a[i:i + batch], gr[i:i + batch], True)
                else:
                    C.conv_update(state, li, a[i:i + batch], gr[i:i + batch], l.k, l.pad, l.stride, True)
            done += min(batch, images - i)
            if time.perf_counter() - t0 >= budget_s and i + batch < images:
                break  # a partial pass: its batches plus one inversion below
        C.invert(state, *DAMPING)
        passes += 1
        if time.perf_counter() - t0 >= budget_s:
            break
    dt = time.perf_counter() - t0
    return done / dt, threads, (f"{done} synthetic images in {passes} pass(es) of up to {images}, "
                                f"batch {batch}, update+invert per pass, torch {torch.__version__} CPU "
                                f"fp32, {threads} thread(s)")


def cpu_e2e_baseline(config, images, batch, budget_s=6.0, threads=None):
    """The reference's end-to-end CPU loop (oracle/cpu_ref_torch.e2e_pass: forward with
    its hooks, Categorical labels, CE backward, update, invert) on a bounded sample of
    the workload's batches; returns (images/s, threads, sample)."""
    from oracle import cpu_ref_torch as C
    if threads is None:
        threads = int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1)
    torch.set_num_threads(threads)
    net = build_model(config, torch.device("cpu"))
    hooked = C.HookedCPU(net)
    rng = np.random.default_rng(0)
    x = torch.from_numpy(rng.random((images, *CONFIGS[config][0].in_shape), dtype=np.float32))
    done, t0 = 0, time.perf_counter()
    C.e2e_pass(hooked, net, x, batch, *DAMPING, max_batches=1)  # warm-up
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < budget_s:
        d, _ = C.e2e_pass(hooked, net, x, batch, *DAMPING,
                          max_batches=max(1, int(budget_s * 2)))
        done += d
    dt = time.perf_counter() - t0
    return done / dt, threads, (f"{done} synthetic images, batch {batch}: forward + Categorical labels + "
                                f"CE backward + update (reference hooks) + invert per group of batches, "
                                f"torch {torch.__version__} CPU fp32, {threads} thread(s)")


def verify_parity(kfac, net, specs, recs, batch, images, world, rank, device, sync, nbatches=2,
                  seed0=1234, ref_factory=None):
    """N > 1 self-check, run after the timed region: is the sharded pass + all-reduce
    the single-device pass of the same global batches (models/curvatures.py:359-363)?

    * every rank runs `nbatches` of its batches through the data-parallel `kfac`
      (alpha = 1 / global batch, ONE all-reduce of the packed triangles, invert);
    * rank 0 regenerates every rank's records (same seeds: synthetic_records is a
      function of (seed, shape) only; a per-rank float64 checksum of the rows used
      guards that), concatenates each global batch in rank order and runs a plain
      single-device KFAC over them;
    * rank 0 compares the reduced factors at rtol 1e-5 (of each factor's max) and the
      L factors at 1e-4 of max|L| (the north-star tolerance; the reduced factors
      differ from the single-device sums in the last bits, which cond(R) amplifies);
    * every rank checks that it holds bit-identical L factors (rank 0's broadcast).
    Returns {"ok": bool, ...} on every rank (the verdict is broadcast)."""
    from bnn_kfac_amd.curvatures import KFAC
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    rows = [min(batch, images - i) for i in range(0, images, batch)][:nbatches]
    starts = [sum(rows[:b]) for b in range(len(rows))]
    kfac.reset()
    for s, n in zip(starts, rows):
        for layer, (a, g) in zip(layers, recs):
            kfac.record[layer] = [a[s:s + n], g[s:s + n]]
        kfac.update(batch_size=n, global_batch_size=n * world)
    kfac.invert(*DAMPING)
    inv = kfac.inv_state
    mine_F = [F_ for layer in layers for F_ in kfac.state[layer]]
    mine_L = [L_ for layer in layers for L_ in inv[layer]]
    sync()
    used = sum(rows)
    csum = torch.tensor([float(sum(t[:used].double().sum() for pair in recs for t in pair))],
                        dtype=torch.float64, device=device)
    sums = [torch.zeros_like(csum) for _ in range(world)]
    dist.all_gather(sums, csum)
    detail = {"batches": len(rows), "global_batch": batch * world, "rows_per_rank": used,
              "tolerance": "factors rtol 1e-5 of max|F|; L atol 1e-4 of max|L|; L bit-identical on all ranks"}
    verdict = torch.zeros(1, dtype=torch.float64, device=device)
    if rank == 0:
        per_rank = [recs]
        ok_sums = True
        for r in range(1, world):
            other = synthetic_records(specs, images, device, seed=seed0 + r)
            other = [(a[:used].clone(), g[:used].clone()) for a, g in other]
            got = float(sum(t.double().sum() for pair in other for t in pair))
            ok_sums &= abs(got - float(sums[r])) <= 1e-9 * max(1.0, abs(got))
            per_rank.append(other)
        ref = (ref_factory or KFAC)(net)
        for s, n in zip(starts, rows):
            for li, layer in enumerate(layers):
                a = torch.cat([pr[li][0][s:s + n] for pr in per_rank])
                g = torch.cat([pr[li][1][s:s + n] for pr in per_rank])
                ref.record[layer] = [a, g]
            ref.update(batch_size=n * world)
        ref.invert(*DAMPING)
        ref_inv = ref.inv_state
        for h in ref.hooks:
            h.remove()
        want_F = [F_ for layer in layers for F_ in ref.state[layer]]
        want_L = [L_ for layer in layers for L_ in ref_inv[layer]]
        err_F = max(float((g - w).abs().max() / w.abs().max().clamp_min(1e-30)) for g, w in zip(mine_F, want_F))
        err_L = max(float((g - w).abs().max() / w.abs().max().clamp_min(1e-30)) for g, w in zip(mine_L, want_L))
        upper = all(bool((torch.triu(L_, 1) == 0).all()) for L_ in mine_L)
        ok = ok_sums and err_F <= 1e-5 and err_L <= 1e-4 and upper
        detail.update({"records_checksum_match": ok_sums, "max_rel_err_factors": err_F,
                       "max_rel_err_L": err_L, "L_lower_triangular": upper})
        verdict.fill_(1.0 if ok else 0.0)
        del ref, per_rank
    # every rank holds the same L factors, bit for bit
    flat = torch.cat([L_.reshape(-1) for L_ in mine_L])
    root = flat.clone()
    dist.broadcast(root, 0)
    same = torch.tensor([1.0 if torch.equal(root, flat) else 0.0], dtype=torch.float64, device=device)
    dist.all_reduce(same, op=dist.ReduceOp.MIN)
    dist.broadcast(verdict, 0)
    detail["identical_L_all_ranks"] = bool(float(same) == 1.0)
    detail["ok"] = bool(float(verdict) == 1.0) and detail["identical_L_all_ranks"]
    return detail


# the factor-product kernel families (profile slots of the library, named as rocprofv3
# names them) that compute each fp32 product as six bf16 MFMA products
BF16X3_KERNELS = ("kfac_factor_tiles_x3", "kfac_factor_syrk3", "kfac_factor_conv_x3", "kfac_factor_conv_x3s",
                  "kfac_factor_conv_x3f", "kfac_factor_channel_x3")


def load_traffic(config):
    """The committed PMC profile of `config`'s single-GPU bench (profiles/summarize.py):
    {"tag", "kernels": {family: {hbm_bytes_per_launch, rocprof_trace, ...}}}, or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{config}.json")
    if not os.path.exists(path):
        return None
    with open(path) as f:
        return json.load(f)


def profiled_steps(N, one_pass, kfac, sync, steps):
    """`steps` more pipelined steps with the library's HIP-event timing on: {kernel
    family: (ms, launches, algorithmic flops, algorithmic bytes)} of every factor-product
    kernel family (one library profile slot each), plus the reduce and the inversion."""
    N.profile_reset()
    N.profile_enable(True)
    for _ in range(steps):
        one_pass()
    kfac.inv_state
    sync()
    N.profile_enable(False)
    out = {name: N.profile_read_work(pid) for pid, name in N.PROF_FACTOR_KERNELS.items()}
    out["reduce"] = N.profile_read(N.PROF_FACTOR_REDUCE)
    out["invert"] = N.profile_read(N.PROF_INVERT)
    N.profile_reset()
    return out


def roofline_of(prof, specs, images, steps, config):
    """The roofline object of the dominant factor-product kernel family (the one that
    took the most time among the library's per-family profile slots) and the per-step
    breakdown, from profiled_steps' timings of `steps` passes of `images` images.
    achieved = that family's OWN algorithmic flops (the library sums K_rows * n (n + 1)
    over the jobs it launched) / its launch time; traffic = the committed rocprofv3
    PMC passes of the same family in this config's bench (profiles/pmc_<config>.json)."""
    fams = {k: v for k, v in prof.items() if k not in ("reduce", "invert")}
    kern = max(fams, key=lambda k: fams[k][0])
    ms, launches, flops, abytes = fams[kern]
    bf16x3 = kern in BF16X3_KERNELS
    achieved = flops / (ms * 1e-3) / 1e12 if ms > 0 else None
    peak = SYRK3_PEAK_TFLOPS if bf16x3 else MFMA_F32_PEAK_TFLOPS
    pmc = load_traffic(config)
    k_pmc = (pmc or {}).get("kernels", {}).get(kern)
    traffic = k_pmc.get("hbm_bytes_per_launch") if k_pmc else None
    roofline = {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                "frac": (achieved / peak) if achieved else None,
                "traffic": traffic,
                "traffic_source": (f"profiles/{pmc.get('tag')}/: rocprofv3 --pmc FETCH_SIZE x{k_pmc.get('fetch_scale', 2):g}"
                                   f" + WRITE_SIZE, mean per {kern} launch of the single-GPU {config} bench "
                                   f"(rocprofv3 kernel trace of that run: {k_pmc.get('rocprof_trace')})")
                                  if k_pmc else None,
                "kernel": kern,
                # (the same rate against the fp32 MFMA peak, the basis of earlier rounds)
                "frac_fp32_peak_basis": (achieved / MFMA_F32_PEAK_TFLOPS) if achieved else None,
                "peak_basis": ("dense bf16 MFMA 2.5 PF / 6 products per fp32 product (fp32-equivalent)"
                               if bf16x3 else "dense fp32 MFMA"),
                "launches": launches,
                "avg_launch_us": 1e3 * ms / max(launches, 1),
                # the family's own work per launch (library profile slot), not the step's
                "flops_per_launch": flops / max(launches, 1),
                "algorithmic_bytes_per_launch": abytes / max(launches, 1)}
    fam_rows = {k: {"ms_per_step": v[0] / steps, "launches_per_step": v[1] / steps,
                    "tflops": (v[2] / (v[0] * 1e-3) / 1e12) if v[0] > 0 else None}
                for k, v in fams.items() if v[1]}
    breakdown = {"factor_tiles_ms_per_step": sum(v[0] for v in fams.values()) / steps,
                 "factor_kernels": fam_rows,
                 "factor_reduce_ms_per_step": prof["reduce"][0] / steps,
                 "invert_ms_per_step": prof["invert"][0] / steps,
                 "factor_flops_per_step_check": sum(v[2] for v in fams.values()) / steps,
                 "factor_flops_per_step_algorithmic": flops_per_image(specs) * images}
    return roofline, breakdown


def other_config(config, device, steps, warmup):
    """A GPU-only line for another BASELINE config on this one GPU (C3 LeNet-5, C5 wide
    MLP): the same pipelined pass + invert loop as the headline (records resident,
    eager_verdict False, one launch per records-held cap), `steps` timed steps after
    `warmup`, then the instrumented repetition for its dominant kernel's roofline."""
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import KFAC
    specs = CONFIGS[config]
    batch, images = SHAPES[(config, 1)]
    net = build_model(config, device)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    kfac = KFAC(net)
    kfac.eager_verdict = False
    kfac.launch_first = 16
    recs = synthetic_records(specs, images, device, seed=1234)
    starts = list(range(0, images, batch))
    views = [[(layer, [a[i:i + batch], g[i:i + batch]]) for layer, (a, g) in zip(layers, recs)]
             for i in starts]
    sizes = [min(batch, images - i) for i in starts]

    def one_pass():
        kfac.reset()
        for batch_views, size in zip(views, sizes):
            for layer, rec in batch_views:
                kfac.record[layer] = rec
            kfac.update(batch_size=size)
        kfac.invert(*DAMPING)

    def sync():
        torch.cuda.synchronize(device)

    for _ in range(warmup):
        one_pass()
    kfac.inv_state
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        one_pass()
    kfac.inv_state  # every verdict read inside the timed region
    sync()
    elapsed = time.perf_counter() - t0
    prof = profiled_steps(N, one_pass, kfac, sync, steps)
    roofline, breakdown = roofline_of(prof, specs, images, steps, config)
    for h in kfac.hooks:
        h.remove()
    del kfac, recs, views
    torch.cuda.empty_cache()
    return {"value": images * steps / elapsed, "unit": "images/s", "ms_per_step": 1e3 * elapsed / steps,
            "steps": steps, "warmup": warmup, "config": config, "batch": batch, "images": images,
            "workload": f"{BASELINE_CONFIG[(config, 1)]}: {NAMES[config]} KFAC factor pass over {images} "
                        f"images (batch {batch}) + invert{DAMPING}, pipelined as the headline",
            "roofline": roofline, "breakdown": breakdown}


EIG_SIZES = (785, 4097)  # the MNIST MLP's layer-1 A factor; the wide MLP's (C5) 4096 + ones


def eig_factor(n, seed=0):
    """A synthetic SPD factor of size n: X X^T / n + 1e-3 I, X ~ N(0, 1) (fp32), the shape
    of a KFAC A factor (a Wishart spectrum)."""
    rng = np.random.default_rng(seed + n)
    X = rng.standard_normal((n, n)).astype(np.float32)
    return torch.from_numpy(X @ X.T / n + 1e-3 * np.eye(n, dtype=np.float32))


def eig_leg(device, sizes=EIG_SIZES, reps=3):
    """BASELINE C5's "HBM-bound eig reported" (models/utilities.py:120-141, get_eigenvalues:
    symeig of every factor): the device eigenvalue path (kfac_syev: tridiagonalisation +
    Sturm multisection, fp64) on one factor per size, timed by the library's HIP events
    on its stream (profile slot KFAC_PROF_SYEV).  `achieved` = the tridiagonalisation's
    algorithmic bytes (each reflector reads and rewrites the trailing rows once,
    sum_k (n - k)^2 x 16 B ~ 16 n^3 / 3) / the call's time.  At n = 785 the rows stay in
    LDS (latency-bound: one grid-wide exchange per reflector); at 4097 they stream from
    HBM."""
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.utilities import symeig
    out = {}
    for n in sizes:
        F = eig_factor(n).to(device)
        symeig([F])  # warm-up (also builds nothing: no caches on this path)
        torch.cuda.synchronize(device)
        N.profile_reset()
        N.profile_enable(True)
        t0 = time.perf_counter()
        for _ in range(reps):
            ev = symeig([F])[0][0]
        torch.cuda.synchronize(device)
        wall = (time.perf_counter() - t0) / reps
        N.profile_enable(False)
        ms, calls, _, abytes = N.profile_read_work(N.PROF_SYEV)
        N.profile_reset()
        ms_call = ms / max(calls, 1)
        gbs = abytes / max(calls, 1) / (ms_call * 1e-3) / 1e9 if ms_call > 0 else None
        out[str(n)] = {"ms": ms_call, "wall_ms": 1e3 * wall, "calls": calls,
                       "algorithmic_bytes": abytes / max(calls, 1),
                       "roofline": {"bound": "hbm" if n > 2000 else "latency", "achieved": gbs,
                                    "peak": HBM_PEAK_GBS, "unit": "GB/s",
                                    "frac": gbs / HBM_PEAK_GBS if gbs else None, "traffic": None,
                                    "kernel": "eig_tridiag (+ eig_bisect)"},
                       "eigvals_checksum": float(ev.sum())}
        del F
    torch.cuda.empty_cache()
    return out


def eig_cpu_baseline(sizes=EIG_SIZES, threads=None, budget_s=6.0):
    """The reference's eigenvalue path on the host cores: torch.symeig's successor
    torch.linalg.eigvalsh (LAPACK syevd) on the same fp32 factors (utilities.py:136-137
    calls symeig on the fp32 KFAC factors), repeated within ~budget_s per size."""
    if threads:
        torch.set_num_threads(threads)
    out = {}
    for n in sizes:
        F = eig_factor(n)
        torch.linalg.eigvalsh(F)
        reps, t0 = 0, time.perf_counter()
        while True:
            torch.linalg.eigvalsh(F)
            reps += 1
            if time.perf_counter() - t0 >= budget_s / len(sizes) or reps >= 50:
                break
        out[str(n)] = {"ms": 1e3 * (time.perf_counter() - t0) / reps, "reps": reps}
    return {"value": out, "unit": "ms per eigenvalue solve", "cores": torch.get_num_threads(),
            "kind": "port", "sample": f"torch {torch.__version__} CPU linalg.eigvalsh (LAPACK syevd) on the "
                                      f"fp32 factor, fp32 as the reference's symeig, per size"}


# ------------------------------------------------------------------ launcher
def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n, argv, cmd=None, check_devices=True, poll_s=0.2):
    """Run `n` rank processes of this script (or of `cmd`) on one node and return the
    worst exit code.  Each child gets RANK = LOCAL_RANK = r, WORLD_SIZE =
    LOCAL_WORLD_SIZE = n, MASTER_ADDR = 127.0.0.1 and one free MASTER_PORT; it sets
    its own device and joins the process group.  The parent makes no HIP call
    (torch.cuda.device_count() does not initialise the runtime on this image), so a
    rank's GPU work never shares a process with another's.  When one rank fails,
    the others are terminated (their exact PIDs)."""
    if check_devices:
        have = torch.cuda.device_count()
        if have < n:
            print(f"bench.py --gpus {n}: only {have} GPU(s) visible on this node; need {n} "
                  f"(one rank per GPU)", file=sys.stderr, flush=True)
            return 2
    port = _free_port()
    cmd = cmd or [sys.executable, os.path.abspath(__file__)] + list(argv)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n),
                   LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0", MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
        procs.append(subprocess.Popen(cmd, env=env))
    codes = [None] * n
    first_bad = 0
    while any(c is None for c in codes):
        for i, p in enumerate(procs):
            if codes[i] is None:
                codes[i] = p.poll()
                if codes[i] not in (None, 0) and not first_bad:
                    first_bad = codes[i] if codes[i] > 0 else 1
        if first_bad:
            for i, p in enumerate(procs):
                if codes[i] is None:
                    p.terminate()
            for i, p in enumerate(procs):
                if codes[i] is None:
                    try:
                        codes[i] = p.wait(timeout=20)
                    except subprocess.TimeoutExpired:
                        p.kill()
                        codes[i] = p.wait()
            break
        time.sleep(poll_s)
    return first_bad


# ------------------------------------------------------------------ one rank
def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    # 50 steps: the timed region ends with the last inversion's drain (~0.5 ms on the
    # MLP, not overlapped by a next pass), 8 % of a 10-step region, <2 % of 50
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--config", default="mlp", choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-rank batch (default: the config's)")
    ap.add_argument("--images", type=int, default=None, help="images per rank per pass")
    ap.add_argument("--strong", action="store_true",
                    help="strong scaling: 65,536 x 64 images in global batches of 65,536 over the N ranks")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-e2e", action="store_true")
    ap.add_argument("--no-serial", action="store_true")
    ap.add_argument("--no-other-configs", action="store_true",
                    help="N = 1 MLP: skip the C3 (LeNet-5) and C5 (wide MLP) lines")
    ap.add_argument("--no-eig", action="store_true",
                    help="N = 1 MLP: skip the eigensolver leg (n = 785, 4097)")
    ap.add_argument("--launch-first", type=int, default=None,
                    help="queued updates in a pass's first SYRK launch (KFAC.launch_first) for both "
                         "loops (default: 16 for the pipelined loop, the library's 1 for the serial one)")
    ap.add_argument("--max-pending", type=int, default=None,
                    help="KFAC.max_pending: inversions with an unread verdict before invert() waits (A/B)")
    ap.add_argument("--defer-mb", type=int, default=None,
                    help="KFAC.defer_bytes in MiB (records a queued launch may hold; A/B)")
    ap.add_argument("--single-buffer", action="store_true",
                    help="KFAC.double_buffer = False (the data stream waits for each "
                         "inversion to have read its factors)")
    ap.add_argument("--host-profile", default=None,
                    help="diagnostic: after the timed region, run --steps more pipelined steps under "
                         "cProfile and write the host-side statistics (tottime) to this file")
    ap.add_argument("--no-parity", action="store_true",
                    help="N > 1: skip the post-timing verification pass (verify_parity)")
    ap.add_argument("--shared-device", action="store_true",
                    help="rehearsal on a 1-GPU box: every rank on device 0, gloo instead of RCCL "
                         "(the line says so in config.parallelism; never a scaling number)")
    argv = sys.argv[1:] if argv is None else argv
    args = ap.parse_args(argv)

    if "WORLD_SIZE" not in os.environ:
        if args.gpus > 1:
            return spawn_ranks(args.gpus, argv, check_devices=not args.shared_device)
        world = 1
    else:
        world = int(os.environ["WORLD_SIZE"])
        if world != args.gpus and not (args.gpus == 1 and world > 1):
            print(f"bench.py: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks",
                  file=sys.stderr, flush=True)
            return 2
    rank = int(os.environ.get("RANK", "0"))
    local = 0 if args.shared_device else int(os.environ.get("LOCAL_RANK", "0"))
    if torch.cuda.device_count() <= local:
        print(f"bench.py rank {rank}: LOCAL_RANK {local} but only {torch.cuda.device_count()} GPU(s) "
              f"visible", file=sys.stderr, flush=True)
        return 2
    shape_key = (args.config, 1 if world == 1 else 2)
    batch, images = workload(args.config, world, args.strong)
    batch = args.batch or batch
    images = args.images or images

    torch.cuda.set_device(local)
    device = torch.device("cuda", local)
    if world > 1:
        if args.shared_device:
            dist.init_process_group("gloo")
        else:
            dist.init_process_group("nccl", device_id=device)
    # all GPU work on one non-default stream
    torch.cuda.set_stream(torch.cuda.Stream(device))

    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import KFAC
    from bnn_kfac_amd.distributed import DistributedKFAC

    others = None
    if world == 1 and args.config == "mlp" and not args.no_other_configs and not args.strong:
        # BASELINE's other single-GPU configs (C5 wide MLP, C3 LeNet-5), GPU-only, in
        # the same run, BEFORE the headline: from an idle GPU the pipelined MLP step
        # takes ~60 steps to settle (0.38 -> 0.34 ms per step in blocks of 20,
        # tools/probe_warm.py, profiles/r05k/), so with these first the headline's
        # warmup and timed steps run on a GPU that is already busy, as in training
        others = {"C5": other_config("wide", device, steps=10, warmup=2),
                  "C3": other_config("lenet", device, steps=20, warmup=2)}
        torch.cuda.empty_cache()
    eig = None
    if world == 1 and args.config == "mlp" and not args.no_eig and not args.strong:
        eig = eig_leg(device)

    specs = CONFIGS[args.config]
    net = build_model(args.config, device)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    kfac = DistributedKFAC(net) if world > 1 else KFAC(net)
    # pipelined passes: the pivot verdict of inversion k is read at the next
    # invert() / inv_state read instead of inside invert() (the library's default,
    # the reference's behaviour), so pass k+1 is queued behind inversion k and
    # overlaps it; every verdict is still read inside the timed region below
    kfac.eager_verdict = False
    # pipelined loop: the pass's queued updates go out as ONE SYRK launch at the flush
    # (launch_first 16 >= the MLP's 15 updates; the records-held cap splits LeNet-5's
    # passes anyway): the inversion of pass k overlaps the host's issue of pass k+1
    # as well as its SYRK.  MLP line, one box, 2 reps: 1.51-1.53e8 vs 1.41e8 img/s at
    # the library default 1; the serial loop keeps 1 (8.6e7 vs 8.0e7 img/s at 16:
    # there the GPU would wait for the host to queue the pass) -- profiles/r03_knobs/
    pipe_launch_first = args.launch_first or 16
    serial_launch_first = args.launch_first or kfac.launch_first
    kfac.launch_first = pipe_launch_first
    if args.single_buffer:
        kfac.double_buffer = False
    if args.defer_mb:
        kfac.defer_bytes = args.defer_mb << 20
    if args.max_pending:
        kfac.max_pending = args.max_pending
    recs = synthetic_records(specs, images, device, seed=1234 + rank)
    starts = list(range(0, images, batch))
    comm = {"ms": 0.0, "n": 0, "timing": False}

    if world > 1:
        # the instrumented repetition times the collective with events on the
        # caller's stream (the collective's own stream is joined into it both ways)
        _allreduce = kfac.allreduce

        def timed_allreduce():
            if not comm["timing"] or not kfac._pending:
                return _allreduce()
            kfac.flush()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            _allreduce()
            e1.record()
            comm.setdefault("events", []).append((e0, e1))
        kfac.allreduce = timed_allreduce

    # the batches' record views, made once: in training the hooks hand KFAC fresh
    # tensors per batch at no cost of its own, so slicing the resident records
    # (~2.7 us of host time per view, 60 per MLP pass) stays out of the timed loop
    views = [[(layer, [a[i:i + batch], g[i:i + batch]]) for layer, (a, g) in zip(layers, recs)]
             for i in starts]
    sizes = [min(batch, images - i) for i in starts]
    record = kfac.record

    def one_pass():
        kfac.reset()
        for batch_views, size in zip(views, sizes):
            for layer, rec in batch_views:
                record[layer] = rec
            kfac.update(batch_size=size)
        kfac.invert(*DAMPING)

    def sync():
        torch.cuda.synchronize(device)
        if world > 1:
            dist.barrier()

    def max_over_ranks(x):
        if world == 1:
            return x
        t = torch.tensor([x], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t)

    # The serial figure first (like the C5 / C3 legs above): the pipelined headline
    # below is then warmed up and timed on a GPU that has been busy with this workload.
    # From idle the GPU's clocks ramp over ~20-30 ms of it (the step 0.39 -> 0.35 ms in
    # blocks of 20 steps; the ramp recurs after 1 s idle: profiles/r05m/), which at
    # K = 20 steps would otherwise be most of the timed region.  The end-to-end leg
    # (torch forward/backward GEMMs) stays after the headline: run before it, it slowed
    # the headline's SYRK (312 vs 295 us per launch, 1.61e8 vs 1.73e8 img/s on one box,
    # profiles/r05p/).
    serial = None
    if not args.no_serial:
        # the caller who runs a pass, inverts on its own stream and reads the result
        # before the next pass (classification_ll_block.py:93-106): no overlap
        kfac.overlap_invert = False
        kfac.launch_first = serial_launch_first
        one_pass()
        kfac.inv_state
        sync()
        t1 = time.perf_counter()
        for _ in range(args.steps):
            one_pass()
            kfac.inv_state
            torch.cuda.synchronize(device)
        sync()
        serial = world * images * args.steps / max_over_ranks(time.perf_counter() - t1)
        kfac.overlap_invert = True
        kfac.launch_first = pipe_launch_first


    for _ in range(args.warmup):
        one_pass()
    kfac.inv_state  # settle the warmup's verdicts
    sync()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        one_pass()
    t_issue = time.perf_counter() - t0  # host time to queue the K steps (diagnostic)
    # inside the timed region: join the inversion worker and read every pending
    # pivot verdict (a singular factor raises here, as the reference's would)
    kfac.inv_state
    sync()
    elapsed = max_over_ranks(time.perf_counter() - t0)

    if args.host_profile:
        import cProfile
        import io
        import pstats
        pr = cProfile.Profile()
        t1 = time.perf_counter()
        pr.enable()
        for _ in range(args.steps):
            one_pass()
        pr.disable()
        t_prof = time.perf_counter() - t1
        kfac.inv_state
        sync()
        out = io.StringIO()
        out.write(f"{args.steps} pipelined steps issued in {1e3 * t_prof / args.steps:.3f} ms/step under cProfile "
                  f"(unprofiled host issue {1e3 * t_issue / args.steps:.3f} ms/step)\n")
        # per step, in microseconds (pstats' own listing rounds to milliseconds)
        st = pstats.Stats(pr).stats
        for key, label in ((3, "cumulative"), (2, "own")):
            out.write(f"\n-- {label} us per step --\n")
            for fn, v in sorted(st.items(), key=lambda kv: -kv[1][key])[:35]:
                out.write(f"{1e6 * v[key] / args.steps:9.1f} us  {v[1] / args.steps:6.1f} calls  "
                          f"{os.path.basename(fn[0])}:{fn[1]}({fn[2]})\n")
        with open(args.host_profile, "w") as f:
            f.write(out.getvalue())

    # Kernel durations: the same K steps again with the library's HIP-event timing
    # on (events recorded around each launch, on its stream).  Kept out of the timed
    # region above because the event packets add ~10 us per launch boundary.
    comm["timing"] = True
    if world > 1:  # the side-stream collective (DistributedKFAC.side_collective) times itself
        kfac.comm_events = comm.setdefault("events", [])
    prof = profiled_steps(N, one_pass, kfac, sync, args.steps)
    comm["timing"] = False
    if world > 1:
        kfac.comm_events = None
    allreduce_ms = None
    if world > 1:
        allreduce_ms = max_over_ranks(sum(a.elapsed_time(b) for a, b in comm.pop("events", []))
                                      / args.steps)

    e2e = None
    if not args.no_e2e and world == 1:
        x = torch.rand(images, *specs[0].in_shape, device=device)
        crit = torch.nn.CrossEntropyLoss()

        def e2e_pass():
            kfac.reset()
            for layer in layers:  # own record lists (the hooks fill them in place)
                record[layer] = [None, None]
            for i in starts:
                logits = net(x[i:i + batch])
                labels = torch.distributions.Categorical(logits=logits).sample()
                loss = crit(logits, labels)
                net.zero_grad()
                loss.backward()
                kfac.update(batch_size=logits.shape[0])
            kfac.invert(*DAMPING)
        e2e_pass()
        kfac.inv_state
        sync()
        t1 = time.perf_counter()
        reps = max(1, args.steps // 2)
        for _ in range(reps):
            e2e_pass()
        kfac.inv_state
        sync()
        e2e = images * reps / (time.perf_counter() - t1)
        del x

    images_total = world * images * args.steps
    value = images_total / elapsed
    ms_per_step = 1e3 * elapsed / args.steps
    roofline, breakdown = roofline_of(prof, specs, images, args.steps, args.config)
    breakdown.update({"allreduce_ms_per_step": allreduce_ms,
                      "host_issue_ms_per_step": 1e3 * t_issue / args.steps,
                      "updates_per_step": len(starts)})


    parity = None
    if world > 1 and not args.no_parity:
        parity = verify_parity(kfac, net, specs, recs, batch, images, world, rank, device, sync)


    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the host's best: every thread count this process may use -- its CPU affinity,
        # its cgroup CPU quota and OMP_NUM_THREADS (the box's per-GPU share) -- timed,
        # the fastest reported (`cores` = its thread count), and 1 thread beside them
        hc = host_cpus()
        quota = int(hc["cgroup_quota_cpus"]) if hc["cgroup_quota_cpus"] else None
        counts = sorted({c for c in (hc["affinity"], hc["omp_num_threads"], quota) if c})
        runs = {c: cpu_baseline(specs, images, batch, threads=c) for c in counts}
        best = max(runs, key=lambda c: runs[c][0])
        v, cores, sample = runs[best]
        v1, _, sample1 = cpu_baseline(specs, images, batch, budget_s=6.0, threads=1)
        cpu = {"value": v, "unit": "images/s", "cores": cores, "kind": "port", "sample": sample,
               "value_by_threads": {str(c): r[0] for c, r in runs.items()},
               "value_1_thread": v1, "sample_1_thread": sample1, "cpu_model": cpu_model(),
               "host_cpus": hc, "logical_cpus_visible": os.cpu_count()}
        if args.config == "mlp":
            # BASELINE C1: the reference's CPU pass at ITS batch (256), and the CPU
            # end-to-end loop beside the GPU's e2e_images_per_s
            vc1, _, samplec1 = cpu_baseline(specs, 60000, 256, budget_s=6.0, threads=cores)
            ve, _, samplee = cpu_e2e_baseline(args.config, 60000, 256, threads=cores)
            cpu.update({"c1_batch256_value": vc1, "c1_batch256_sample": samplec1,
                        "e2e_value": ve, "e2e_sample": samplee})
        # the other configs' CPU baselines: the same op sequence on a bounded sample of
        # their workload, at the thread count the headline's baseline found best
        for name, oc in (others or {}).items():
            v_o, c_o, s_o = cpu_baseline(CONFIGS[oc["config"]], oc["images"], oc["batch"], budget_s=6.0,
                                         threads=cores)
            oc["cpu_baseline"] = {"value": v_o, "unit": "images/s", "cores": c_o, "kind": "port", "sample": s_o}
        if eig is not None:
            eig_cpu = eig_cpu_baseline(threads=cores)
            for n, e in eig.items():
                e["cpu_baseline_ms"] = eig_cpu["value"][n]["ms"]
            eig_cpu["value"] = {n: v["ms"] for n, v in eig_cpu["value"].items()}
            eig["cpu_baseline"] = eig_cpu

    if rank == 0:
        cfg = BASELINE_CONFIG[shape_key]
        out = {"metric": METRIC, "value": value, "unit": "images/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms_per_step,
               "higher_is_better": True, "scaling": "strong" if args.strong else "weak",
               "vs_baseline": None, "dtype": "f32",
               "metric_variant": ("pipelined: inversion k overlaps pass k+1 (eager_verdict=False); "
                                  "serial_images_per_s = images / (T_pass + T_invert), the "
                                  "reference scripts' order"),
               "data": "synthetic (resident U[0,1) activations, N(0,1) output-gradient records)",
               "config": {"workload": f"{cfg}: {NAMES[args.config]} KFAC factor pass over {images} "
                                      f"images/rank (batch {batch}/rank, global batch {batch * world}) "
                                      f"+ invert{DAMPING}",
                          "baseline_config": cfg + (" strong" if args.strong else ""),
                          "global_batch": batch * world,
                          "images_per_rank": images,
                          "parallelism": f"dp{world}" + (" (shared device, gloo: rehearsal, not a "
                                                         "scaling number)" if args.shared_device else ""),
                          "inversion": ("sharded" if getattr(kfac, "_sharded_last", False)
                                        else "replicated"),
                          "launch_first": {"pipelined": pipe_launch_first, "serial": serial_launch_first}},
               "roofline": roofline, "cpu_baseline": cpu, "breakdown": breakdown,
               "allreduce_ms_per_step": allreduce_ms,
               # N > 1: the sharded pass + all-reduce vs a single-device recompute of the
               # same global batches (verify_parity, after the timed region); N = 1: null
               "parity": None if parity is None else parity["ok"], "parity_detail": parity,
               "serial_images_per_s": serial, "e2e_images_per_s": e2e,
               # BASELINE C3 / C5 on this GPU, same loop (GPU-only; N = 1 MLP runs)
               "other_configs": others,
               # BASELINE C5's eig leg: kfac_syev values at the MLP's 785 and the wide 4097
               "eig": eig}
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
