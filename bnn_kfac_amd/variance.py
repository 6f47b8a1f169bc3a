"""Sampling-free predictive variance with Kronecker-factored posteriors.

Replaces the per-layer `J_i @ torch.kron(Q_i, H_i) @ J_i.t()` loops of
sampling_free/classification/classification_ll_block.py:114-170 and
sampling_free/regression/regression_ll_block.py:120-140 with one grouped device
contraction (libkfac_hip `kfac_kron_quadform`) that never forms the Kronecker
product.  The Jacobians J themselves stay host-side PyTorch autograd, exactly as
the reference builds them (sampling_free/utils.py:221-226).
"""
from __future__ import annotations

from typing import Iterable, List, Sequence, Tuple

import numpy as np
import torch
from torch import Tensor

from . import _native as N


def gradient(y: Tensor, x: Tensor, grad_outputs: Tensor = None) -> Tensor:
    """dy/dx @ grad_outputs (sampling_free/utils.py:221-226)."""
    if grad_outputs is None:
        grad_outputs = torch.ones_like(y)
    return torch.autograd.grad(y, [x], grad_outputs=grad_outputs, create_graph=True,
                               retain_graph=True, allow_unused=True)[0]


def layer_jacobian(output: Tensor, layer: torch.nn.Module, grad_outputs: Tensor) -> Tensor:
    """J_i = cat([flatten(dW), flatten(db)]) (classification_ll_block.py:128-130)."""
    g = [torch.flatten(gradient(output, p, grad_outputs)) for p in layer.parameters()]
    return torch.cat(g, dim=0)


def kron_quadform(terms: Sequence[Tuple[Tensor, Tensor, Tensor]], lower: bool = True,
                  abs_sum: bool = True, per_term: bool = False):
    """sum_l |J_l kron(K1_l, K2_l) J_l^T| for rows of J_l (shape (nb, nA*nG) or (nA*nG,)).

    terms: [(J_l, K1_l, K2_l)], K1 (nA x nA), K2 (nG x nG), J in the reference's flat
    order a*nG + g.  `lower` marks K1/K2 as lower-triangular (Cholesky factors from
    KFAC.invert) so their zero blocks are skipped.  Returns out (nb,) fp32 and, if
    per_term, the raw per-layer values (L, nb).
    """
    if not terms:
        raise ValueError("no terms")
    Js = []
    nb = None
    for J, K1, K2 in terms:
        J2 = J.detach()
        J2 = J2.reshape(1, -1) if J2.dim() == 1 else J2
        if J2.stride(-1) != 1:
            J2 = J2.contiguous()
        if nb is None:
            nb = J2.shape[0]
        elif J2.shape[0] != nb:
            raise ValueError("all terms need the same number of rows")
        Js.append(J2)
    device = Js[0].device
    out = torch.empty(nb, dtype=torch.float32, device=device)
    v = torch.empty(len(terms), nb, dtype=torch.float32, device=device) if per_term else None
    keep = []
    groups = []
    for li, ((_, K1, K2), J2) in enumerate(zip(terms, Js)):
        nA, nG = K1.shape[0], K2.shape[0]
        if J2.shape[1] != nA * nG:
            raise ValueError(f"J has {J2.shape[1]} columns, kron(K1, K2) needs {nA * nG}")
        for t, what in ((J2, "J"), (K1, "K1"), (K2, "K2")):
            N.require_device(t, what)
        K1c = K1.detach() if K1.stride(-1) == 1 else K1.detach().contiguous()
        K2c = K2.detach() if K2.stride(-1) == 1 else K2.detach().contiguous()
        keep.extend([K1c, K2c])
        q = N.QuadJob()
        q.J, q.ldJ, q.nA, q.nG = J2.data_ptr(), J2.stride(0) if nb > 1 else nA * nG, nA, nG
        q.K1, q.ld1, q.K2, q.ld2 = K1c.data_ptr(), K1c.stride(0), K2c.data_ptr(), K2c.stride(0)
        q.lower1 = q.lower2 = int(lower)
        q.v = v[li].data_ptr() if per_term else 0
        groups.append(q)
    # the C-ABI groups up to 8 terms per launch; fold larger models in chunks
    if len(groups) <= 8:
        N.kron_quadform(groups, nb, abs_sum, out)
    else:
        acc = torch.zeros(nb, dtype=torch.float32, device=device)
        for g0 in range(0, len(groups), 8):
            part = torch.empty(nb, dtype=torch.float32, device=device)
            N.kron_quadform(groups[g0:g0 + 8], nb, abs_sum, part)
            acc += part
        out = acc
    return (out, v) if per_term else out


def layer_jacobians(output: Tensor, layers: Sequence[torch.nn.Module], grad_outputs: Tensor) -> List[Tensor]:
    """[J_i] for several layers from ONE backward pass: the same vectors as the
    reference's per-parameter `gradient` calls (classification_ll_block.py:128-130,
    sampling_free/utils.py:221-226), which each run a full backward."""
    params = [p for layer in layers for p in layer.parameters()]
    grads = torch.autograd.grad(output, params, grad_outputs=grad_outputs, retain_graph=True,
                                allow_unused=True)
    out, k = [], 0
    for layer in layers:
        n = len(list(layer.parameters()))
        out.append(torch.cat([torch.flatten(g) for g in grads[k:k + n]], dim=0))
        k += n
    return out


def kfac_predictive_std(kfac, output: Tensor, grad_outputs: Tensor, layers: Iterable = None,
                        per_layer: bool = False):
    """The reference's `pred_std` for one test batch (classification_ll_block.py:118-132):
    sum over KFAC layers of |J_i kron(L_A, L_G) J_i^T|, J_i the gradient of
    `output` weighted by `grad_outputs` w.r.t. the layer's [W, b]."""
    if layers is None:
        layers = [m for m in list(kfac.model.modules())[1:] if m in kfac.state]
    layers = list(layers)
    terms = []
    for layer, J in zip(layers, layer_jacobians(output, layers, grad_outputs)):
        LA, LG = kfac.inv_state[layer]
        terms.append((J, LA, LG))
    res = kron_quadform(terms, lower=True, abs_sum=True, per_term=per_layer)
    if per_layer:
        return float(res[0][0]), res[1][:, 0]
    return float(res[0])


def per_sample_predictive_std(kfac, x: Tensor, layers: Iterable = None, chunk: int = 256) -> Tensor:
    """Predictive std of every sample of `x` as the reference computes it for a test
    batch of ONE image (classification_ll_block.py:114-135 / the noise loop 147-165):
    p = softmax(net(x_b)), grad_outputs = one-hot(argmax p), J_l = d(go . p)/d[W_l, b_l],
    std_b = sum_l |J_l kron(L_A, L_G) J_l^T|.

    Per-sample Jacobians come from ONE vmapped gradient per chunk (torch.func), and
    the whole chunk is contracted by a single kfac_kron_quadform launch (nb rows per
    layer) instead of a Python loop of single-image backward passes.  Returns (N,) fp32.
    """
    from collections import OrderedDict

    from torch.func import functional_call, grad, vmap
    model = kfac.model
    if layers is None:
        layers = [m for m in list(model.modules())[1:] if m in kfac.state]
    layers = list(layers)
    names = {id(p): n for n, p in model.named_parameters()}
    pnames = [[names[id(p)] for p in layer.parameters()] for layer in layers]
    # KFAC's module hooks (record capture) must not fire inside the functorch
    # transforms: suspend every module hook for this call, then restore the exact
    # hook dictionaries
    kinds = ("_forward_hooks", "_forward_pre_hooks", "_backward_hooks", "_backward_pre_hooks")
    saved = [(m, [getattr(m, k) for k in kinds]) for m in model.modules()]
    for m, _ in saved:
        for k in kinds:
            setattr(m, k, OrderedDict())
    try:
        return _per_sample_std(kfac, model, layers, pnames, x, chunk, functional_call, grad, vmap)
    finally:
        for m, dicts in saved:
            for k, d in zip(kinds, dicts):
                setattr(m, k, d)


def _per_sample_std(kfac, model, layers, pnames, x, chunk, functional_call, grad, vmap):
    flat = [n for group in pnames for n in group]
    params = {n: p.detach() for n, p in model.named_parameters()}
    buffers = {n: b for n, b in model.named_buffers()}

    def score(theta, xb):
        full = dict(params)
        full.update(theta)
        p = torch.softmax(functional_call(model, (full, buffers), (xb.unsqueeze(0),)), dim=1)[0]
        go = (p == p.max()).to(p.dtype)  # one-hot argmax (a comparison: no gradient through it)
        return (go.detach() * p).sum()

    jac = vmap(grad(score), in_dims=(None, 0))
    out = []
    for c0 in range(0, x.shape[0], chunk):
        g = jac({n: params[n] for n in flat}, x[c0:c0 + chunk])
        terms = []
        for layer, group in zip(layers, pnames):
            J = torch.cat([g[n].reshape(g[n].shape[0], -1) for n in group], dim=1)
            LA, LG = kfac.inv_state[layer]
            terms.append((J, LA, LG))
        out.append(kron_quadform(terms, lower=True, abs_sum=True))
    return torch.cat(out)


def argmax_grad_outputs(pred_mean: Tensor) -> Tensor:
    """grad_outputs[:, idx] = 1 with idx = argmax per row, set for EVERY row
    (classification_ll_block.py:119-121 semantics)."""
    idx = np.argmax(pred_mean.detach().cpu().numpy(), axis=1)
    grad_outputs = torch.zeros_like(pred_mean)
    grad_outputs[:, idx] = 1
    return grad_outputs


def entropy_bits(pred_std: float) -> float:
    """0.5 * log2(2 pi e var) (classification_ll_block.py:134-135)."""
    return float(0.5 * np.log2(2 * np.e * np.pi * pred_std))


def regression_inverse_factors(kfac, N_data: float, tau: float) -> List[Tuple[Tensor, Tensor]]:
    """pinv(N (q + tau I)) and pinv(N (h + tau I)) for every state entry
    (regression_ll_block.py:128-133).  q + tau I is SPD for tau > 0, so the
    pseudo-inverse is the inverse; computed by the fp64 device path."""
    jobs, outs = [], []
    device = None
    for layer, (q, h) in kfac.state.items():
        pair = []
        for F_ in (q, h):
            N.require_device(F_, "state", layer)
            out = torch.empty_like(F_, memory_format=torch.contiguous_format)
            jobs.append(N.invert_job(F_, out, float(N_data), float(N_data) * float(tau), N.OUT_INVERSE))
            pair.append(out)
            device = F_.device
        outs.append(tuple(pair))
    info = N.invert(jobs, device)
    if bool((info.cpu() != 0).any()):
        raise np.linalg.LinAlgError("SVD did not converge")
    return outs
