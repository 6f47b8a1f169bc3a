"""Time the sampling-free predictive-variance path.

Network: the reference's BaseNet_15k shapes (conv 1->5 k5, pool, conv 5->10 k5, pool,
fc 160->80, fc 80->10; KFAC factors A 26/126/161/81, G 5/10/80/10), random init,
factors accumulated by KFAC over synthetic batches and inverted at (0.04, 200).

Per test batch (classification_ll_block.py:114-132): softmax output, argmax
grad_outputs, per-layer Jacobian by autograd (row 13, PyTorch), then
sum_l |J_l kron(L_A, L_G) J_l^T|:
  gpu_e2e     : autograd on the GPU + kfac_kron_quadform (no kron materialised)
  gpu_quadform: the device contraction alone, all layers of one batch in one call
  cpu_ref     : the reference's op sequence on the host (autograd + torch.kron +
                J @ H @ J^T), same inputs, torch CPU fp32 on this host's threads
Prints one JSON line.
"""
import json
import os
import sys
import time

import numpy as np
import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402
from bnn_kfac_amd.variance import (argmax_grad_outputs, kron_quadform, layer_jacobian,  # noqa: E402
                                   layer_jacobians, per_sample_predictive_std)


def basenet15k():
    torch.manual_seed(0)
    return nn.Sequential(nn.Conv2d(1, 5, 5), nn.ReLU(), nn.MaxPool2d(2), nn.Conv2d(5, 10, 5), nn.ReLU(),
                         nn.MaxPool2d(2), nn.Flatten(), nn.Linear(160, 80), nn.ReLU(), nn.Linear(80, 10))


def pred_std_terms(net, layers, inv_state, x):
    """One backward pass for all layers' Jacobians (variance.layer_jacobians)."""
    out = torch.softmax(net(x), dim=1)
    go = argmax_grad_outputs(out)
    return [(J.unsqueeze(0), *inv_state[l]) for l, J in zip(layers, layer_jacobians(out, layers, go))]


def main():
    dev = torch.device("cuda:0")
    batch = int(os.environ.get("VAR_BATCH", "256"))
    nbatch = int(os.environ.get("VAR_NBATCH", "20"))
    net = basenet15k().to(dev)
    kfac = KFAC(net)
    crit = nn.CrossEntropyLoss()
    g = torch.Generator(device=dev).manual_seed(0)
    for _ in range(8):
        x = torch.rand(1024, 1, 28, 28, device=dev, generator=g)
        logits = net(x)
        y = torch.distributions.Categorical(logits=logits).sample()
        net.zero_grad()
        crit(logits, y).backward()
        kfac.update(batch_size=x.shape[0])
    kfac.invert(0.04, 200)
    layers = [m for m in list(net.modules())[1:] if m in kfac.state]
    tests = [torch.rand(batch, 1, 28, 28, device=dev, generator=g) for _ in range(nbatch)]

    # GPU end to end
    for x in tests[:2]:
        kron_quadform(pred_std_terms(net, layers, kfac.inv_state, x))
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    vals = []
    for x in tests:
        vals.append(kron_quadform(pred_std_terms(net, layers, kfac.inv_state, x)))
    torch.cuda.synchronize()
    gpu_e2e = (time.perf_counter() - t0) / nbatch

    # device contraction alone
    terms = pred_std_terms(net, layers, kfac.inv_state, tests[0])
    terms = [(J.detach(), A, G) for J, A, G in terms]
    for _ in range(3):
        kron_quadform(terms)
    torch.cuda.synchronize()
    reps = 200
    t0 = time.perf_counter()
    for _ in range(reps):
        kron_quadform(terms)
    torch.cuda.synchronize()
    gpu_q = (time.perf_counter() - t0) / reps

    # per-sample std (the reference's noise loop: test batches of ONE image), vmapped
    xs = torch.rand(2048, 1, 28, 28, device=dev, generator=g)
    per_sample_predictive_std(kfac, xs[:256])
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    per_sample_predictive_std(kfac, xs)
    torch.cuda.synchronize()
    gpu_ps_us = (time.perf_counter() - t0) / xs.shape[0] * 1e6

    # the reference's op sequence on the host, same weights, factors and inputs
    torch.set_num_threads(int(os.environ.get("OMP_NUM_THREADS", "0")) or (os.cpu_count() or 1))
    net_c = basenet15k()
    net_c.load_state_dict({k: v.cpu() for k, v in net.state_dict().items()})
    layers_c = [m for m in list(net_c.modules())[1:] if isinstance(m, (nn.Conv2d, nn.Linear))]
    inv_c = {lc: tuple(t.cpu() for t in kfac.inv_state[lg]) for lc, lg in zip(layers_c, layers)}
    ncpu = max(2, min(nbatch, 4))
    t0 = time.perf_counter()
    tq = 0.0
    ref_vals = []
    for x in tests[:ncpu]:
        xc = x.cpu()
        out = torch.softmax(net_c(xc), dim=1)
        go = argmax_grad_outputs(out)
        s = 0.0
        for l in layers_c:
            J = layer_jacobian(out, l, go).unsqueeze(0).detach()
            q0 = time.perf_counter()
            H = torch.kron(*inv_c[l])
            s += torch.abs(J @ H @ J.t()).item()
            tq += time.perf_counter() - q0
        ref_vals.append(s)
    cpu_ref = (time.perf_counter() - t0) / ncpu
    cpu_q = tq / ncpu
    # one image per "batch" on the host (the noise loop), a few images
    t0 = time.perf_counter()
    nimg = 8
    for b in range(nimg):
        out1 = torch.softmax(net_c(xs[b:b + 1].cpu()), dim=1)
        go1 = argmax_grad_outputs(out1)
        s1 = 0.0
        for l in layers_c:
            J = layer_jacobian(out1, l, go1).unsqueeze(0).detach()
            s1 += torch.abs(J @ torch.kron(*inv_c[l]) @ J.t()).item()
    cpu_ps_us = (time.perf_counter() - t0) / nimg * 1e6
    got = np.array([float(v) for v in vals[:ncpu]])
    rel = float(np.max(np.abs(got - np.array(ref_vals)) / np.abs(np.array(ref_vals))))
    print(json.dumps({
        "workload": f"BaseNet_15k predictive std, {nbatch} test batches of {batch}",
        "gpu_e2e_ms_per_batch": gpu_e2e * 1e3, "gpu_quadform_ms_per_batch": gpu_q * 1e3,
        "cpu_ref_ms_per_batch": cpu_ref * 1e3, "cpu_ref_kron_quadform_ms_per_batch": cpu_q * 1e3,
        "gpu_per_sample_us": gpu_ps_us, "cpu_ref_per_sample_us": cpu_ps_us,
        "cpu_threads": torch.get_num_threads(), "cpu_batches": ncpu,
        "max_rel_diff_vs_cpu_ref": rel}))


if __name__ == "__main__":
    main()
