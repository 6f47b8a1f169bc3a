"""Test double for the device kernels so the HOST logic (operand descriptors,
alpha/beta bookkeeping, packed state, all-reduce, damping parsing) can be tested
on a CPU-only machine.  It reads the same ctypes job descriptors the C ABI
receives and applies the oracle's formula to the raw host memory they point at.
Never used by the product path (bnn_kfac_amd raises without a GPU)."""
import ctypes

import numpy as np


UPDATES = []  # per kfac_factor_update call: nseg of each job
ACC = {}      # deferred-reduction accumulators: slab-range pointer -> n x n partial sum
SLAB_BYTES = 64 * 64 * 4  # a slab range starting at split s0 sits s0 tiles into the buffer


def _view(ptr, count):
    return np.ctypeslib.as_array((ctypes.c_float * max(count, 1)).from_address(ptr))[:count]


def fake_factor_update(jobs, device):
    """kfac_factor_update: F = beta F + alpha X~^T X~, or with a deferred-reduction
    accumulator (modelled as one n x n split) acc = acc_beta acc + alpha X~^T X~."""
    from bnn_kfac_amd import _native as N
    UPDATES.append([max(1, j.nseg) for j in jobs])
    for j in jobs:
        op = j.x
        assert op.layout == N.ROWMAJOR, "test double handles row-major operands only"
        if j.nseg > 1:  # multi-batch job: seg_ptrs is a (host) int64 table of batch bases
            bases = np.ctypeslib.as_array((ctypes.c_int64 * j.nseg).from_address(j.seg_ptrs))
        else:
            bases = [op.ptr]
        # a ragged last batch (x.last_rows) enters with weight rows / last_rows
        rows = [op.rows] * len(bases)
        if j.nseg > 1 and 0 < op.last_rows < op.rows:
            rows[-1] = op.last_rows
        Xs = []
        for b, r in zip(bases, rows):
            Xb = _view(int(b), r * op.ld).reshape(r, op.ld)[:, :op.cols].astype(np.float64)
            Xs.append(Xb * np.sqrt(op.rows / r))
        X = np.concatenate(Xs)
        if op.has_ones:
            ones = np.concatenate([np.full((r, 1), np.sqrt(op.rows / r)) for r in rows])
            X = np.concatenate([X, ones], axis=1)
        n = op.cols + op.has_ones
        if j.acc:
            # (modelled per slab range: ACC[acc pointer] = that range's n x n partial sum)
            assert j.acc_splits == 1
            new = j.alpha * (X.T @ X)
            if j.acc_beta != 0.0:
                new = new + j.acc_beta * ACC[j.acc].astype(np.float64)
            ACC[j.acc] = new.astype(np.float32)
            continue
        F = _view(j.F, n * j.ldF).reshape(n, j.ldF)
        new = j.alpha * (X.T @ X)
        if j.beta != 0.0:
            new = new + j.beta * F[:, :n].astype(np.float64)
        F[:, :n] = new.astype(np.float32)


def fake_accum_plan(jobs):
    # (one split; the device plan's bytes: lower-triangle tiles x splits x one 64 x 64 slab)
    def tiles(n):
        t = (n + 63) // 64
        return t * (t + 1) // 2
    return [(1, tiles(j.x.cols + j.x.has_ones) * SLAB_BYTES) for j in jobs]


FLUSHES = []
FLUSH_STREAMS = []  # per flush: the raw stream it was issued on (None: the caller's)


def fake_factor_flush(jobs, device, stream=None):
    """kfac_factor_flush: F = beta F + alpha acc."""
    FLUSHES.append(len(jobs))
    FLUSH_STREAMS.append(stream)
    for j in jobs:
        n = j.x.cols + j.x.has_ones
        stride = j.acc_stride or j.acc_splits
        used = [p for p in ACC if j.acc <= p < j.acc + stride * SLAB_BYTES]
        A = sum(ACC[p].astype(np.float64) for p in used)
        for p in used:  # (the cycle's ranges are consumed: the next cycle writes fresh ones)
            del ACC[p]
        F = _view(j.F, n * j.ldF).reshape(n, j.ldF)
        new = j.alpha * A
        if j.beta != 0.0:
            new = new + j.beta * F[:, :n].astype(np.float64)
        F[:, :n] = new.astype(np.float32)


def install(monkeypatch):
    from bnn_kfac_amd import _native as N
    # (accumulators of an earlier test live at host addresses a later test's buffers
    # may reuse: every test starts with none)
    ACC.clear()
    monkeypatch.setattr(N, "require_device", lambda t, what, owner=None: None)
    monkeypatch.setattr(N, "factor_update", fake_factor_update)
    monkeypatch.setattr(N, "factor_accum_plan", fake_accum_plan)
    monkeypatch.setattr(N, "factor_flush", fake_factor_flush)


def _tri_rows(n):
    return [(i, i * (i + 1) // 2) for i in range(n)]


def fake_tri_pack(jobs, packed):
    """kfac_tri_pack on host memory."""
    P = packed.numpy() if hasattr(packed, "numpy") else packed
    for j in jobs:
        F = _view(j.F, j.n * j.ldF).reshape(j.n, j.ldF) if j.n else None
        for i, off in _tri_rows(j.n):
            P[j.offset + off:j.offset + off + i + 1] = F[i, :i + 1]


def fake_tri_unpack(jobs, packed, mode):
    """kfac_tri_unpack on host memory (mode 0 mirrors, 1 zeroes the upper triangle)."""
    P = packed.numpy() if hasattr(packed, "numpy") else packed
    for j in jobs:
        F = _view(j.F, j.n * j.ldF).reshape(j.n, j.ldF) if j.n else None
        for i, off in _tri_rows(j.n):
            F[i, :i + 1] = P[j.offset + off:j.offset + off + i + 1]
            if mode == 0:
                F[:i, i] = F[i, :i]
            else:
                F[i, i + 1:j.n] = 0.0


def fake_invert(jobs, device, inputs_read=None):
    """kfac_invert (OUT_INV_CHOL): L = cholesky(inv(scale (F+F^T)/2 + shift I)) in fp64;
    info = 1 for a factor that is not positive definite."""
    import torch
    info = []
    for j in jobs:
        F = _view(j.F, j.n * j.ldF).reshape(j.n, j.ldF)[:, :j.n].astype(np.float64)
        R = j.scale * (F + F.T) / 2 + j.shift * np.eye(j.n)
        out = _view(j.out, j.n * j.ldo).reshape(j.n, j.ldo)
        try:
            out[:, :j.n] = np.linalg.cholesky(np.linalg.inv(R)).astype(np.float32)
            info.append(0)
        except np.linalg.LinAlgError:
            info.append(1)
    return torch.tensor(info, dtype=torch.int32)


class HostEvent:
    def __init__(self, *a, **k):
        pass

    def record(self, stream=None):
        pass

    def query(self):
        return True

    def synchronize(self):
        pass


class _HostStream:
    def wait_stream(self, other):
        pass

    def wait_event(self, ev):
        pass


class _NoStream:
    def __init__(self, stream=None):
        pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


class HostRawEvent:
    """Test double of N.RawEvent (host work is synchronous: always complete)."""
    def __init__(self, device=None, ordering=False):
        self.handle = 0
        self.ordering = ordering

    def close(self):
        pass

    def record(self, stream):
        pass

    def wait_on(self, stream):
        pass

    def query(self):
        return True

    def synchronize(self):
        pass


def fake_invert_pipelined(jobs, device, info_host, order, inputs_read, done, main, side, side_stream=None):
    info = fake_invert(jobs, device)
    info_host.copy_(info)
    return info


def install_cuda_stubs(kfac_list=()):
    """Stand-ins for the torch.cuda stream / event calls of KFAC.invert (run with
    overlap_invert False) so the plain single-device path runs on host memory; the
    verdict readback of each KFAC in `kfac_list` uses an unpinned buffer."""
    import torch
    from bnn_kfac_amd import _native as N
    N.RawEvent = HostRawEvent
    N.invert_pipelined = fake_invert_pipelined
    N.stream_handle = lambda device: 0
    stream = _HostStream()
    torch.cuda.current_stream = lambda device=None: stream
    torch.cuda.stream = _NoStream
    torch.cuda.Event = HostEvent
    for k in kfac_list:
        k.overlap_invert = False
        k._pinned_info = lambda info: torch.empty(info.numel(), dtype=torch.int32)
        k._pinned_host = lambda n: torch.empty(n, dtype=torch.int32)


def install_distributed(kfac=None):
    """Host doubles for the collectives' device kernels (and the sharded inversion's
    verdict readback on `kfac`)."""
    from bnn_kfac_amd import _native as N
    N.require_device = lambda t, what, owner=None: None
    N.factor_update = fake_factor_update
    N.factor_accum_plan = fake_accum_plan
    N.factor_flush = fake_factor_flush
    N.tri_pack = fake_tri_pack
    N.tri_unpack = fake_tri_unpack
    N.invert = fake_invert
    if kfac is not None:
        kfac._readback = lambda info: (HostEvent(), info.clone())
