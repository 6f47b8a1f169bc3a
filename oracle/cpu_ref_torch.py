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
* end to end (classification_ll_block.py:93-106): forward with the reference's
  hooks recording the layer inputs (curvatures.py:319-320) and grad_output * B
  (:322-323), a Categorical label draw, cross-entropy backward, the update above
  per batch, then invert.
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


class HookedCPU:
    """The reference's hooks on a CPU model (curvatures.py:310-323): forward pre-hook
    keeps the input, backward hook keeps grad_output[0] * batch."""

    def __init__(self, model):
        self.layers = [m for m in model.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
        self.record = {m: [None, None] for m in self.layers}
        for m in self.layers:
            m.register_forward_pre_hook(self._save_input)
            m.register_full_backward_hook(self._save_output)

    def _save_input(self, module, inp):
        self.record[module][0] = inp[0]

    def _save_output(self, module, grad_input, grad_output):
        self.record[module][1] = grad_output[0] * grad_output[0].size(0)

    def update(self, state):
        for i, m in enumerate(self.layers):
            a, g = self.record[m]
            if isinstance(m, torch.nn.Conv2d):
                conv_update(state, i, a.detach(), g.detach(), m.kernel_size, m.padding, m.stride,
                            m.bias is not None)
            else:
                linear_update(state, i, a.detach(), g.detach(), m.bias is not None)


def e2e_pass(hooked: HookedCPU, model, x: torch.Tensor, batch: int, add: float, multiply: float,
             max_batches: int = None):
    """One pass of classification_ll_block.py:93-106 on the CPU; returns (images, inv)."""
    state, done = {}, 0
    crit = torch.nn.CrossEntropyLoss()
    for bi, i in enumerate(range(0, x.shape[0], batch)):
        if max_batches is not None and bi >= max_batches:
            break
        xb = x[i:i + batch]
        logits = model(xb)
        labels = torch.distributions.Categorical(logits=logits).sample()
        loss = crit(logits, labels)
        model.zero_grad()
        loss.backward()
        hooked.update(state)
        done += xb.shape[0]
    return done, invert(state, add, multiply)
