"""CPU baseline: the reference's KFAC op sequence on torch CPU (fp32, MKL/OpenMP).

TEST/BENCH INFRASTRUCTURE ONLY (bench.py's `cpu_baseline` leg and tests).  This is
a restatement ("port") of `models/curvatures.py:325-398` op for op, so that the
reference's own CPU cost can be timed on the GPU box's host cores, where the
reference itself does not travel:

* update  (curvatures.py:345-363): f = [a^T; 1^T]; A = mm(f, f^T) / B;
  G = mm(g^T, g) / B; first batch assigns, later batches `+=`.
* conv update (curvatures.py:341-343,352-353): f = unfold(x, k, padding, stride)
  permuted to (C*k*k, B*L) (+ ones row); b = g.permute(1,0,2,3) as (C_out, B*L);
  A = mm(f, f^T) / (B*L), G = mm(b, b^T) / (B*L).
* invert  (curvatures.py:374-398): R = s**0.5 * F + diag(n**0.5); R = (R + R^T)/2;
  L = R.inverse().cholesky()  (torch.linalg.inv + torch.linalg.cholesky, the
  non-deprecated names of the same LAPACK getrf/getri + potrf calls).
"""
from __future__ import annotations

import torch


def linear_update(state: dict, name, a: torch.Tensor, g_rec: torch.Tensor, has_bias: bool):
    f = a.t()
    if has_bias:
        f = torch.cat([f, torch.ones_like(f[:1])], dim=0)
    A = torch.mm(f, f.t()) / float(f.shape[1])
    b = g_rec.t()
    G = torch.mm(b, b.t()) / float(b.shape[1])
    if name in state:
        state[name][0] += A
        state[name][1] += G
    else:
        state[name] = [A, G]


def conv_update(state: dict, name, x: torch.Tensor, g_rec: torch.Tensor, kernel, padding, stride,
                has_bias: bool):
    f = torch.nn.functional.unfold(x, kernel, padding=padding, stride=stride)
    f = f.permute(1, 0, 2).contiguous().view(f.shape[1], -1)
    if has_bias:
        f = torch.cat([f, torch.ones_like(f[:1])], dim=0)
    A = torch.mm(f, f.t()) / float(f.shape[1])
    b = g_rec.permute(1, 0, 2, 3).contiguous().view(g_rec.shape[1], -1)
    G = torch.mm(b, b.t()) / float(b.shape[1])
    if name in state:
        state[name][0] += A
        state[name][1] += G
    else:
        state[name] = [A, G]


def invert(state: dict, add=0.0, multiply=1.0) -> dict:
    inv = {}
    n, s = float(add), float(multiply)
    for name, (first, second) in state.items():
        out = []
        for F in (first, second):
            R = s ** 0.5 * F + torch.diag(F.new(F.shape[0]).fill_(n ** 0.5))
            R = (R + R.t()) / 2.0
            out.append(torch.linalg.cholesky(torch.linalg.inv(R)))
        inv[name] = tuple(out)
    return inv
