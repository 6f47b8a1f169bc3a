"""Eigen/Kronecker helpers of the KFAC path (models/utilities.py:120-159, 387-409).

`get_eigenvalues` / `get_eigenvectors` keep the reference's signatures and output
layout; the eigensolves run on the device (libkfac_hip `kfac_syev`, fp64 Jacobi)
instead of the removed `torch.symeig`.
"""
from __future__ import annotations

from typing import Dict, List

import torch
from torch import Tensor
from torch.nn import Module

from . import _native as N


def kron(a: Tensor, b: Tensor) -> Tensor:
    r"""Kronecker product, index (i*p + k, j*q + l) = a[i,j] b[k,l] (utilities.py:387-409).

    >>> a = torch.tensor([[1, 2], [3, 4]])
    >>> b = torch.tensor([[0, 5], [6, 7]])
    >>> kron(a, b)
    tensor([[ 0,  5,  0, 10],
            [ 6,  7, 12, 14],
            [ 0, 15,  0, 20],
            [18, 21, 24, 28]])
    """
    return (a[:, None, :, None] * b[None, :, None, :]).reshape(a.size(0) * b.size(0),
                                                               a.size(1) * b.size(1))


def symeig(factors: List[Tensor], eigenvectors: bool = False, symmetrize: bool = True):
    """Device eigendecomposition of a list of square fp32 factors (grouped launch).

    Returns [(eigvals fp64 ascending, eigvecs fp32 or None)] — `torch.symeig`'s
    ascending order, computed on (F + F^T)/2.
    """
    if not factors:
        return []
    device = factors[0].device
    jobs, outs = [], []
    for F_ in factors:
        N.require_device(F_, "factor")
        n = F_.shape[0]
        evals = torch.empty(n, dtype=torch.float64, device=device)
        evecs = torch.empty(n, n, dtype=torch.float32, device=device) if eigenvectors else None
        j = N.EigJob()
        j.F, j.ldF, j.n = F_.data_ptr(), F_.stride(0), n
        j.evals, j.evecs, j.ldv = evals.data_ptr(), N.ptr(evecs), n
        jobs.append(j)
        outs.append((evals, evecs))
    info = N.syev(jobs, device)
    if bool((info.cpu() != 0).any()):
        raise RuntimeError("symmetric eigensolver did not converge")
    return outs


def get_eigenvalues(factors: List, verbose: bool = False) -> Tensor:
    """utilities.py:120-141: for each [A, G]: ger(eig(A), eig(G)).view(-1); for a
    diagonal factor: factor.view(-1); concatenated.  Eigenvalues fp32 like the
    reference's symeig output (computed in fp64 on device)."""
    pairs = [f for f in factors if len(f) == 2]
    flat = [f for pair in pairs for f in pair]
    eig = iter(symeig(flat))
    out = []
    for factor in factors:
        if len(factor) == 2:
            la = next(eig)[0].float()
            lg = next(eig)[0].float()
            out.append(torch.outer(la, lg).contiguous().view(-1))
        else:
            out.append(factor.contiguous().view(-1))
    return torch.cat(out) if out else torch.zeros(0)


def get_eigenvectors(factors: Dict[Module, List[Tensor]]) -> Dict[Module, tuple]:
    """utilities.py:144-159: eigenvectors of xxt + xxt^T and ggt + ggt^T (ascending)."""
    flat = []
    for xxt, ggt in factors.values():
        flat.extend([xxt + xxt.t(), ggt + ggt.t()])
    res = symeig(flat, eigenvectors=True)
    out = {}
    for i, layer in enumerate(factors.keys()):
        out[layer] = (res[2 * i][1], res[2 * i + 1][1])
    return out
