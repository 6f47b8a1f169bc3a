"""Test double for the device kernels so the HOST logic (operand descriptors,
alpha/beta bookkeeping, packed state, all-reduce, damping parsing) can be tested
on a CPU-only machine.  It reads the same ctypes job descriptors the C ABI
receives and applies the oracle's formula to the raw host memory they point at.
Never used by the product path (bnn_kfac_amd raises without a GPU)."""
import ctypes

import numpy as np


def _view(ptr, count):
    return np.ctypeslib.as_array((ctypes.c_float * max(count, 1)).from_address(ptr))[:count]


def fake_factor_update(jobs, device):
    from bnn_kfac_amd import _native as N
    for j in jobs:
        op = j.x
        assert op.layout == N.ROWMAJOR, "test double handles row-major operands only"
        X = _view(op.ptr, op.rows * op.ld).reshape(op.rows, op.ld)[:, :op.cols].astype(np.float64)
        if op.has_ones:
            X = np.concatenate([X, np.ones((op.rows, 1))], axis=1)
        n = op.cols + op.has_ones
        F = _view(j.F, n * j.ldF).reshape(n, j.ldF)
        new = j.alpha * (X.T @ X)
        if j.beta != 0.0:
            new = new + j.beta * F[:, :n].astype(np.float64)
        F[:, :n] = new.astype(np.float32)


def install(monkeypatch):
    from bnn_kfac_amd import _native as N
    monkeypatch.setattr(N, "require_device", lambda t, what, owner=None: None)
    monkeypatch.setattr(N, "factor_update", fake_factor_update)
