"""Drop-in `curvatures.KFAC` for MI355X.

Mirrors the reference's public interface (models/curvatures.py:17-144 `Curvature`,
:277-405 `KFAC`): same constructor arguments and checks, same hooks, `record`,
`state[layer] = [A, G]`, `inv_state[layer] = (L_A, L_G)` keyed by the module
objects in `model.modules()` order, same damping-argument handling and error
behaviour.  The arithmetic runs in libkfac_hip.so (hand-written gfx950 kernels):

* `update`  -> ONE grouped fp32-MFMA launch (+ one reduce) for all layers' A and G
  (curvatures.py:325-365), Conv2d through an implicit im2col (no F.unfold copy).
* `invert`  -> fp64 blocked potrf + trtri on device, grouped over all factors
  (curvatures.py:367-398), one host sync to read the pivot status.

All factors of a model live in ONE packed fp32 device buffer (state tensors are
views into it), so a data-parallel pass needs exactly one all-reduce
(bnn_kfac_amd.distributed).
"""
from __future__ import annotations

import copy
import os
from abc import ABC, abstractmethod
from typing import Any, List, NamedTuple, Union

import numpy as np
import torch
from torch import Tensor
from torch.nn import Module, Sequential

from . import _native as N

SUPPORTED = ['Linear', 'Conv2d', 'MultiheadAttention']


class Curvature(ABC):
    """Base class (models/curvatures.py:17-144): layer selection, state dicts,
    sampling and checkpointing."""

    def __init__(self, model: Union[Module, Sequential], layer_types: Union[List[str], str] = None):
        # curvatures.py:38-65
        self.model = model
        self.model_state = copy.deepcopy(model.state_dict())
        self.layer_types = list()
        if isinstance(layer_types, str):
            self.layer_types.append(layer_types)
        elif isinstance(layer_types, list):
            if layer_types:
                self.layer_types.extend(layer_types)
            else:
                self.layer_types.extend(SUPPORTED)
        elif layer_types is None:
            self.layer_types.extend(SUPPORTED)
        else:
            raise TypeError
        for _type in self.layer_types:
            assert _type in SUPPORTED
        self.state = dict()
        self.inv_state = dict()

    # `state` reads and writes first complete any reduction an implementation
    # deferred (KFAC keeps a data pass's split-K partials on the device and reduces
    # them into the factors once; see KFAC.flush).
    @property
    def state(self):
        self.flush()
        return self._state

    @state.setter
    def state(self, value):
        self.flush()
        self._state = value

    # `inv_state` reads first settle the verdict of a pending inversion (see
    # KFAC.invert: the device's pivot check is read back asynchronously, so invert()
    # does not stall the host on the GPU).  Writes never wait.
    @property
    def inv_state(self):
        self._check_inverse()
        return self._inv_state

    @inv_state.setter
    def inv_state(self, value):
        self._inv_state = value

    def _check_inverse(self):
        pass

    def flush(self):
        """Complete deferred work so that `state` holds every update so far."""

    @staticmethod
    def _replace(sample: Tensor, weight: Tensor, bias: Tensor = None):
        """Add a sampled offset to a layer's parameters, bias = last column
        (curvatures.py:67-82)."""
        if bias is not None:
            bias_sample = sample[:, -1].contiguous().view(*bias.shape)
            bias.data.add_(bias_sample)
            sample = sample[:, :-1]
        weight.data.add_(sample.contiguous().view(*weight.shape))

    @abstractmethod
    def update(self, *args: Any, **kwargs: Any):
        raise NotImplementedError

    @abstractmethod
    def invert(self, add: Union[float, list, tuple] = 0., multiply: Union[float, list, tuple] = 1.):
        raise NotImplementedError

    @abstractmethod
    def sample(self, layer: Module) -> Tensor:
        raise NotImplementedError

    def sample_and_replace(self):
        """curvatures.py:117-129 (Linear/Conv2d; MultiheadAttention is rejected at construction)."""
        self.model.load_state_dict(self.model_state)
        for layer in self.model.modules():
            if layer.__class__.__name__ in self.layer_types:
                if layer.__class__.__name__ in ['Linear', 'Conv2d']:
                    _sample = self.sample(layer)
                    self._replace(_sample, layer.weight, layer.bias)

    # ---- checkpointing (curvatures.py:132-144).  The reference pickles the whole
    # model with Module objects as dict keys; here the file holds tensors keyed by
    # the module's qualified name (loadable with weights_only=True) and `load`
    # restores the weights into self.model.
    def _names(self):
        return {m: name for name, m in self.model.named_modules()}

    def save(self, filename):
        names = self._names()
        # per-layer values are [A, G] / (L_A, L_G) (KFAC), tuples (INF) or one tensor (EFB)
        def keep(v):
            return list(v) if isinstance(v, (list, tuple)) else v

        torch.save({'state': {names[k]: keep(v) for k, v in self.state.items()},
                    'inv_state': {names[k]: keep(v) for k, v in self.inv_state.items()},
                    'model': self.model.state_dict()}, filename)
        print('Writting %s complete!\n' % filename)

    def load(self, filename):
        blob = torch.load(filename, weights_only=True)
        modules = dict(self.model.named_modules())
        self.model.load_state_dict(blob['model'])
        self.state = {modules[k]: list(v) if isinstance(v, list) else v
                      for k, v in blob['state'].items()}
        self.inv_state = {modules[k]: tuple(v) if isinstance(v, list) else v
                          for k, v in blob['inv_state'].items()}
        print('Loading %s complete!\n' % filename)


# bytes of one 64 x 64 fp32 partial tile: a slab range starting at split s0 of an
# accumulator starts s0 tiles into it (kfac_factor_job.acc_stride)
_SLAB_BYTES = 64 * 64 * 4

# stream priority of the inversion side streams (-1 high; 0 normal measured within the
# box spread in rounds 4 and 5)
_INV_STREAM_PRIO = -1

# stream-ordering events without the system-scope fence (KFAC._event): MLP line
# 1.942-1.954e8 vs 1.912-1.940e8 img/s with every event fenced, 3 alternating reps,
# LeNet-5 equal (profiles/r05bb/)
_ORDERING_EVENTS = True


# The inversion side streams, one pair per device for the whole process: a KFAC object
# made after another (a new model, a new epoch's object) takes the same HIP streams.  New
# streams per object measured the second object's LeNet-5 line at 1.03e7 instead of
# 1.53e7 img/s (tools/other_probe.py twice): with more streams than the device's hardware
# queues (GPU_MAX_HW_QUEUES), a new side stream can share its queue with the caller's
# stream, and the inversion then no longer runs beside the next pass.
_SIDE_STREAMS = {}


def _shared_side_streams(device):
    pair = _SIDE_STREAMS.get(device.index)
    if pair is None:
        pair = _SIDE_STREAMS[device.index] = [torch.cuda.Stream(device=device, priority=_INV_STREAM_PRIO)
                                              for _ in range(2)]
    return pair


def _same_shapes(f, g):
    """Two fast-path templates of the same record signature (layers, shapes, strides)."""
    return all(a[:7] == b[:7] for a, b in zip(f[1], g[1])) and len(f[1]) == len(g[1])


class _Pending(NamedTuple):
    """An inversion whose pivot verdict is not read yet."""
    done: Any            # torch.cuda.Event after the verdict's copy to `host`
    host: Tensor         # pinned int32, one per job (0 = positive definite)
    layers: list         # layers of the inversion, two jobs (A, G) each
    target: dict         # the inv_state dict the layers' factors went into
    outs: list           # the L factors (kept alive until ordered after)
    on_side: bool        # issued on a side stream (the caller's stream must wait)


class KFAC(Curvature):
    r"""Kronecker-factored Fisher (models/curvatures.py:277-405) on MI355X.

    For each Linear/Conv2d layer: Q = E[a a^T] (input, + bias ones row) and
    H = E[g g^T] (output gradients scaled by the batch size), accumulated as a sum
    of per-batch means over `update` calls.
    """

    def __init__(self, model: Union[Module, Sequential], layer_types: Union[List[str], str] = None):
        super().__init__(model, layer_types)
        self.hooks = list()
        self.record = dict()
        for layer in model.modules():
            if layer.__class__.__name__ in self.layer_types:
                if layer.__class__.__name__ in ['Linear', 'Conv2d']:
                    self.record[layer] = [None, None]
                    self.hooks.append(layer.register_forward_pre_hook(self._save_input))
                    # the reference's legacy module backward hook (curvatures.py:315) is a
                    # hook on the grad_fn of the layer's own last op (addmm / convolution):
                    # registered here the same way, from a forward hook, without the
                    # deprecated API.  An in-place activation after the layer
                    # (nn.ReLU(inplace=True), torchvision style) leaves that node intact,
                    # so grad_output[0] is dL/d(out) as in the reference; a full backward
                    # hook wraps the output in a view that such an op breaks at backward.
                    self.hooks.append(layer.register_forward_hook(self._hook_output))
                elif layer.__class__.__name__ == 'MultiheadAttention':
                    raise NotImplementedError
        self._packed = None      # flat fp32 device buffer holding every factor
        self._packed_views = {}  # layer -> (A view, G view)
        # Two packed buffers, alternating per data pass (reset()): an overlapped
        # inversion reads pass k's factors while pass k+1 accumulates into the other
        # buffer, so the caller's stream never waits for an inversion to have read its
        # inputs; the buffer's next writer (the flush of pass k+2) waits for that
        # inversion's inputs-read event instead (long complete by then).
        self.double_buffer = True
        self._alt_packed, self._alt_views = None, {}
        self._buf_read = {}      # packed buffer data_ptr -> inputs-read event of its inversion
        self._layer_list = list(self.record)
        # Deferred execution (flush() completes it; every `state` read flushes):
        # * queued updates: update() resolves each batch's factor jobs and keeps the
        #   records alive (no copy); up to `defer_batches` updates are then launched
        #   together, row-major factors as ONE multi-batch MFMA job each (K walks all
        #   queued batches in place), so a pass costs ~one launch instead of one per batch;
        # * deferred reduction (kfac_factor_flush): the launches keep each factor's
        #   split-K partial tiles in device accumulators; the reduce into `state` runs
        #   once, when the state is next read (invert / save / `state` / all-reduce).
        self.defer_reduce = True
        self.defer_batches = 64
        # queued updates keep their records alive until their launch (the reference
        # frees them after each update): the queue is also launched once the records
        # it holds reach this many bytes, so a wide or conv model's activations are
        # not retained beyond ~this much (MLP batch of 4096: 17 MB per update; LeNet-5
        # batch of 1024: ~35 MB; the wide MLP: 281 MB).  Round 5, same box: 512 MiB +4 %
        # on LeNet-5 (9 launches per pass instead of 15), the wide MLP equal within 0.3 %
        # (two updates per launch instead of one); 1 GiB +6 % on LeNet-5 but -1.6 % on
        # the wide MLP (3-update launches)
        self.defer_bytes = 512 << 20
        self._queue_bytes = 0
        self._queue = []         # per queued update: (jobs, operand pointers, kept records,
                                 # their _version, device, merge key)
        # launch sizes: the first launch of a pass takes `launch_first` queued updates,
        # each later one twice as many (up to defer_batches; defer_bytes caps them
        # too).  1: the GPU starts on a pass while the host is still issuing it.  16
        # (a pass of <= 16 updates = one launch at the flush) measured +1.5 % on the
        # pipelined MLP line, +2.7 % LeNet-5, +0.4 % wide, but -12 % on the serial
        # pass-then-invert loop the reference's scripts run (the host's issue of the
        # pass is no longer overlapped): kept at 1.
        self.launch_first = 1    # (property: also restarts the doubling)
        self._fast = None        # job templates of the last slow-path update (see _remember)
        self._fast_alt = []      # this cycle's other valid templates (other batch shapes)
        self._fast_cache = {}    # packed buffer data_ptr -> templates onto its views (cycle starts)
        # device buffers of the accumulators: two, taken in turn by cycles whose reduce
        # ran on an inversion side stream (reduce_on_side), so the next pass writes one
        # while that reduce still reads the other; `_acc_reads`: buffer data_ptr -> the
        # event after its side reduce, waited for before the buffer is written again
        self._acc_bufs = [None, None]
        self._acc_par = 0
        self._acc_reads = {}
        self._acc_map = None     # F pointer -> (acc pointer, splits) of the pending cycle
        self._acc_live = set()   # F pointers already written in the pending cycle
        self._acc_flush = None   # flush jobs of the pending cycle (None: nothing pending)
        self._acc_device = None
        self._info_pool = []     # free pinned int32 readback buffers of the pivot checks
        self._event_pool = {}    # device index -> settled torch.cuda.Events (no event creation per invert)
        self._inv_older = []     # earlier inversions whose verdict is not read yet (in order)
        self._inv_pending = None  # _Pending of the last inversion until its verdict is settled
        self.overlap_invert = True  # invert() on a side stream (see invert)
        # eager_verdict (default, the reference's behaviour): invert() waits for its own
        # pivot check and raises LinAlgError itself, as the reference's invert does
        # (curvatures.py:393-396).  False (opt-in, bench.py): the verdict is settled at
        # the next inv_state read or invert(), so the next data pass is queued behind
        # the inversion without a host sync and overlaps it.
        self.eager_verdict = True
        # eager_verdict False: inversions whose verdict may stay unread (and whose
        # factors stay queued) before invert() waits for the oldest one
        self.max_pending = 2
        # one launch for the groups of a queued flush (full batches + short last one);
        # off by default: measured neutral to 2 % slower on the MLP line
        self.merge_launches = False
        # invert() of a pass whose reduction is still deferred runs that reduce on the
        # inversion's side stream, ahead of the inversion, instead of on the caller's
        # stream: the next pass's SYRK launch follows the last one directly (latency-
        # bound inversions only, overlap_invert on)
        self.reduce_on_side = True
        self._inv_streams = {}    # device index -> side streams

    def reset(self):
        """Forget the accumulated factors (start a new data pass); device buffers are kept."""
        self._queue = []
        self._queue_bytes = 0
        self._launch_at = self.launch_first
        self._fast = None
        self._fast_alt = []
        self._acc_flush = self._acc_map = None
        self._state = dict()
        self.inv_state = dict()
        if self.double_buffer and self._packed is not None:
            self._packed, self._packed_views, self._alt_packed, self._alt_views = (
                self._alt_packed, self._alt_views, self._packed, self._packed_views)
            if self._packed is None:
                self._packed_views = {}

    def _await_readers(self, stream=None):
        """Order the caller's (or the given) stream after the inversion that read the
        current packed buffer, before that buffer is written or handed out."""
        buf = self._packed
        if buf is None or not self._buf_read:
            return
        ev = self._buf_read.pop(buf.data_ptr(), None)
        if ev is not None:
            # (an event the host already sees complete needs no wait packet on the stream)
            if not (isinstance(ev, N.RawEvent) and ev.query()):
                self._wait(ev, stream, buf.device)
            self._pool_event(buf.device, ev)  # the wait captured its record: reusable

    def flush(self):
        """Launch queued updates, then reduce the pending accumulators into the
        factors (async; one reduce launch).  Afterwards the caller's stream is ordered
        after any inversion still reading the factors (`state` hands them out)."""
        if getattr(self, "_queue", None):
            self._launch_queue()
        self._launch_at = getattr(self, "launch_first", 1)
        jobs = getattr(self, "_acc_flush", None)
        if jobs:
            self._acc_flush = self._acc_map = None
            self._end_cycle(jobs)
        if getattr(self, "_buf_read", None):
            self._await_readers()

    def _end_cycle(self, jobs):
        """Reduce the cycle's accumulators into the factors (one launch, on the
        caller's stream, after any inversion still reading the target buffer)."""
        self._await_readers()
        N.factor_flush(jobs, self._acc_device)

    # curvatures.py:319-323
    def _save_input(self, module, input):
        self.record[module][0] = input[0]

    def _save_output(self, module, grad_input, grad_output):
        self.record[module][1] = grad_output[0] * grad_output[0].size(0)

    def _hook_output(self, module, input, output):
        """Forward hook: the backward hook of this call goes on the output's grad_fn
        (what torch's legacy register_backward_hook does; no grad_fn -> no record)."""
        fn = output.grad_fn if isinstance(output, Tensor) else None
        if fn is not None:
            fn.register_hook(lambda grad_input, grad_output: self._save_output(module, grad_input,
                                                                                grad_output))

    # ------------------------------------------------------------------ update
    def _layers(self):
        """KFAC'd layers in modules() order (curvatures.py:334-337).  Only layers
        hooked at construction have records, so the list is fixed then."""
        return self._layer_list

    @staticmethod
    def _operands(layer, forward: Tensor, backward: Tensor):
        """Operand descriptors replacing curvatures.py:341-356's unfold/permute/t()."""
        N.require_device(forward, "input", layer)
        N.require_device(backward, "output gradient", layer)
        has_bias = layer.bias is not None
        if layer.__class__.__name__ == 'Conv2d':
            if isinstance(layer.padding, str):
                raise TypeError(f"unfold() padding must be a tuple of ints, got {layer.padding!r}")
            # only data pointers are read (no detach()); the records themselves are kept
            # when already contiguous, so later updates can take the fast path
            x, g = forward, backward
            if x.dim() != 4:
                raise RuntimeError(f"Conv2d KFAC expects a 4-D (B,C,H,W) input, got {tuple(x.shape)}")
            if not x.is_contiguous():
                x = x.contiguous()
            if not g.is_contiguous():
                g = g.contiguous()
            opA = N.patch_operand(x, layer.kernel_size, layer.padding, layer.stride, has_bias)
            opG = N.channel_operand(g)
            keep = (x, g)
        else:
            # only data pointers are read: no detach() needed
            a, g = forward, backward
            da, dg = a.dim(), g.dim()
            if da != 2 or dg != 2:
                if da > 2 or dg > 2:
                    raise RuntimeError("t() expects a tensor with <= 2 dimensions, but self is "
                                       f"{max(da, dg)}D")
                a = a.reshape(1, -1) if da == 1 else a
                g = g.reshape(1, -1) if dg == 1 else g
            if a.stride(1) != 1:
                a = a.contiguous()
            if g.stride(1) != 1:
                g = g.contiguous()
            opA = N.rowmajor_operand(a, has_bias)
            opG = N.rowmajor_operand(g, False)
            keep = (a, g)
        nA = opA.cols + opA.has_ones
        nG = opG.cols
        return opA, opG, nA, nG, keep

    @property
    def launch_first(self) -> int:
        return self._launch_first

    @launch_first.setter
    def launch_first(self, value: int):
        self._launch_first = int(value)
        self._launch_at = self._launch_first  # queue length that triggers the next launch

    def _alpha(self, op: N.Operand) -> float:
        """Per-batch mean: 1/cols (curvatures.py:349,356); an empty batch gives
        0 * inf = nan like the reference's 0/0."""
        return 1.0 / float(op.rows) if op.rows else float("inf")

    def _ensure_packed(self, sizes, device):
        """One flat buffer for all factors, views in modules() order."""
        total = sum(nA * nA + nG * nG for _, nA, nG in sizes)
        if self._packed is not None and self._packed.numel() == total and self._packed.device == device:
            return
        self._await_readers()  # the buffer dropped here may still be read by an inversion
        buf = torch.empty(total, dtype=torch.float32, device=device)
        views, off = {}, 0
        for layer, nA, nG in sizes:
            A = buf[off:off + nA * nA].view(nA, nA)
            off += nA * nA
            G = buf[off:off + nG * nG].view(nG, nG)
            off += nG * nG
            views[layer] = (A, G)
        self._packed, self._packed_views = buf, views
        # fast-path templates onto a dropped buffer's views can never match again
        alt = self._alt_packed.data_ptr() if self._alt_packed is not None else None
        self._fast_cache = {k: v for k, v in self._fast_cache.items() if k == alt}

    def _target(self, layer, nA, nG, device):
        """(A, G, beta): where this update writes and whether it accumulates."""
        if layer in self._state:
            A, G = self._state[layer]
            own = self._packed_views.get(layer)
            if own is not None and own[0] is A and own[1] is G:
                return A, G, 1.0  # our own packed views: shapes/layout known
            for F_, n in ((A, nA), (G, nG)):
                if F_.shape != (n, n):
                    raise RuntimeError(f"state of {layer} has shape {tuple(F_.shape)}, update gives {n}x{n}")
                N.require_device(F_, "state", layer)
                if F_.stride(1) != 1:
                    raise RuntimeError("KFAC state factors must be row-major")
            return A, G, 1.0
        A, G = self._packed_views[layer]
        self._state[layer] = [A, G]
        return A, G, 0.0

    def update(self, batch_size: int):
        """Accumulate this batch's factors for every selected layer
        (curvatures.py:325-365; `batch_size` is unused there too)."""
        if self.defer_reduce:
            fast = self._fast
            if fast is not None:
                entry = self._fast_entry(fast)
                if entry is None and self._fast_alt:
                    entry = self._fast_other()
                if entry is not None:
                    self._enqueue(entry)
                    return
            elif not self._state and self._packed is not None:
                entry = self._fast_begin()
                if entry is not None:
                    self._enqueue(entry)
                    return
        cycle_start = not self._state
        prepared = []
        for layer in self._layers():
            forward, backward = self.record[layer]
            if forward is None or backward is None:
                raise AttributeError(f"'NoneType' object has no attribute 'data': no forward/backward "
                                     f"recorded for {layer}")
            prepared.append((layer,) + self._operands(layer, forward, backward))
        if not prepared:
            return
        device = prepared[0][5][0].device
        if any(layer not in self._state for layer, *_ in prepared):
            self._ensure_packed([(p[0], p[3], p[4]) for p in prepared], device)
        jobs, keep = [], []
        for layer, opA, opG, nA, nG, kept in prepared:
            A, G, beta = self._target(layer, nA, nG, device)
            jobs.append(N.factor_job(opA, A, self._alpha(opA), beta))
            jobs.append(N.factor_job(opG, G, self._alpha(opG), beta))
            keep.extend(kept)
        if not self.defer_reduce:
            self._await_readers()
            N.factor_update(jobs, device)
            return
        self._remember(prepared, jobs, device, cycle_start)
        # merge key: the fast path's job templates when later updates can reuse them
        # (they differ from `jobs` only in beta and pointers), else this update alone
        key = self._fast[2] if self._fast is not None else tuple(jobs)
        self._enqueue((tuple(jobs), tuple(j.x.ptr for j in jobs), keep,
                       [t._version for t in keep], device, key, None))

    # Fast path: a later update whose records have the same shapes, strides, dtype and
    # device as the last slow-path one, and whose targets are still the same `state`
    # entries, reuses that update's job templates (beta 1: the factors now exist) and
    # only reads the records' data pointers.
    @staticmethod
    def _signature(t):
        return t.shape, t.stride(), t.dtype, t.device

    def _remember(self, prepared, jobs, device, cycle_start=False):
        old = self._fast
        self._fast = None
        spec = []
        for layer, _opA, _opG, _nA, _nG, kept in prepared:
            forward, backward = self.record[layer]
            if kept[0] is not forward or kept[1] is not backward:
                return  # a reshaped / made-contiguous record: stay on the slow path
            if forward.dtype != backward.dtype or forward.device != backward.device:
                return
            lst = self._state[layer]
            # (shapes, strides, dtype, device index: _fast_entry compares them field by
            # field, cheapest first; the signature of _signature, unpacked)
            spec.append((layer, forward.shape, backward.shape, forward.stride(), backward.stride(),
                         forward.dtype, forward.get_device(), lst, lst[0], lst[1]))
        tmpl, tmpl0 = [], []
        for j in jobs:
            t = N.FactorJob.from_buffer_copy(j)
            t.beta = 1.0
            tmpl.append(t)
            t = N.FactorJob.from_buffer_copy(j)
            t.beta = 0.0
            tmpl0.append(t)
        # bytes of the records one fast-path update keeps queued (the signatures fix them)
        nbytes = sum(t.numel() * t.element_size() for layer, *_ in prepared for t in self.record[layer])
        fast = self._fast = (getattr(self, "_scale", 1.0), spec, tuple(tmpl), device, tuple(tmpl0), nbytes)
        # the templates of other batch shapes stay usable this cycle (same state lists)
        if old is not None and old[1][0][7] is spec[0][7]:
            self._fast_alt = [f for f in [old] + self._fast_alt if not _same_shapes(f, fast)][:3]
        # templates onto this packed buffer's own views start later cycles on it
        # (_fast_begin); kept per buffer, one per batch shape, the cycle's first update
        # shape first
        views = self._packed_views
        buf = self._packed
        if buf is not None and all(views.get(e[0], (None, None))[0] is e[8] and views[e[0]][1] is e[9]
                                   for e in spec):
            lst = [f for f in self._fast_cache.get(buf.data_ptr(), []) if not _same_shapes(f, fast)]
            lst.insert(0 if cycle_start else len(lst), fast)
            self._fast_cache[buf.data_ptr()] = lst[:4]

    def _fast_entry(self, fast, begin=False):
        scale, spec, tmpl, device, tmpl0, nbytes = fast
        if getattr(self, "_scale", 1.0) != scale:
            return None
        record, state = self.record, self._state
        ptrs, keep, versions = [], [], []
        for layer, shp_f, shp_b, str_f, str_b, dtype, dev, lst, A, G in spec:
            forward, backward = record[layer]
            if forward is None or backward is None:
                return None
            if (forward.shape != shp_f or backward.shape != shp_b or forward.dtype != dtype
                    or backward.dtype != dtype or forward.stride() != str_f or backward.stride() != str_b
                    or forward.get_device() != dev or backward.get_device() != dev):
                return None
            if begin:
                v = self._packed_views.get(layer)
                if v is None or v[0] is not A or v[1] is not G:
                    return None
            elif state.get(layer) is not lst or lst[0] is not A or lst[1] is not G:
                return None
            ptrs += (forward.data_ptr(), backward.data_ptr())
            keep += (forward, backward)
            versions += (forward._version, backward._version)
        return tmpl0 if begin else tmpl, tuple(ptrs), keep, versions, device, tmpl, nbytes

    def _fast_other(self):
        """An update of another batch shape seen this cycle (the pass's short last
        batch): its template becomes the primary one."""
        for i, f in enumerate(self._fast_alt):
            entry = self._fast_entry(f)
            if entry is not None:
                self._fast_alt[i] = self._fast
                self._fast = f
                return entry
        return None

    def _fast_begin(self):
        """The first update of a cycle (empty state, after reset()) on a packed buffer a
        slow-path update already wrote: a cached template onto the buffer's views whose
        record signature matches creates the state entries (as _target does) and queues
        the update with the template's beta-0 jobs; the buffer's other templates are
        re-bound to the new state lists for the rest of the cycle."""
        cached = self._fast_cache.get(self._packed.data_ptr())
        if not cached:
            return None
        for i, f in enumerate(cached):
            entry = self._fast_entry(f, begin=True)
            if entry is None:
                continue
            state = self._state
            lists = {}
            for e in f[1]:
                lists[e[0]] = state[e[0]] = [e[8], e[9]]
            rebound = []
            for g in [f] + cached[:i] + cached[i + 1:]:
                spec = [e[:7] + (lists[e[0]], e[8], e[9]) if e[0] in lists else e for e in g[1]]
                rebound.append(g[:1] + (spec,) + g[2:])
            self._fast, self._fast_alt = rebound[0], rebound[1:]
            cached[:] = rebound
            return entry
        return None

    def _enqueue(self, entry):
        """Queue one update: (jobs, operand pointers, records kept alive, their
        _version, device, merge key)."""
        queue = self._queue
        if queue and queue[0][4] is not entry[4] and queue[0][4] != entry[4]:
            self._launch_queue()
        self._queue.append(entry)
        nbytes = entry[6]
        self._queue_bytes += (nbytes if nbytes is not None
                              else sum(t.numel() * t.element_size() for t in entry[2]))
        # launch sizes double from `launch_first` up to defer_batches (the records held
        # are capped by defer_bytes): a function of the update count only, so the
        # launches' K-splits, and with them the factors' fp32 summation order, are the
        # same on every run
        if len(self._queue) >= max(1, self.defer_batches) or self._queue_bytes >= self.defer_bytes:
            self._launch_queue()
        elif len(self._queue) >= self._launch_at:
            self._launch_at *= 2
            self._launch_queue()

    def _launch_queue(self):
        """Launch the queued updates: consecutive updates with the same job templates
        and operand alignment become one multi-batch job per factor (row-major: K
        walks the batches; Conv2d im2col / channel-major: the images walk them)."""
        queue, self._queue = self._queue, []
        self._queue_bytes = 0
        for _jobs, _ptrs, keep, versions, _dev, _key, _nbytes in queue:
            for t, v in zip(keep, versions):
                if t._version != v:
                    raise RuntimeError(
                        "a KFAC record was modified in place after update() and before its "
                        "queued factor update ran; clone it, or set kfac.defer_batches = 1")
        device = queue[0][4]
        groups, start = [], 0
        align = [tuple(p % 16 for p in e[1]) for e in queue]
        for i in range(1, len(queue) + 1):
            if i == len(queue) or queue[i][5] is not queue[start][5] or align[i] != align[start]:
                groups.append(queue[start:i])
                start = i
        align = {id(e): a for e, a in zip(queue, align)}
        # a pass's short last batch joins the batches before it as the ragged last
        # batch of their multi-batch jobs (x.last_rows): one launch instead of two
        ragged = [False] * len(groups)
        i = 0
        while i + 1 < len(groups):
            if len(groups[i + 1]) == 1 and self._ragged_ok(groups[i], groups[i + 1][0], align):
                groups[i] = groups[i] + groups[i + 1]
                del groups[i + 1]
                ragged[i] = True
            i += 1
        tables = []
        launches = []
        for group, rag in zip(groups, ragged):
            tmpl = group[0][0]
            jobs = []
            for k, t in enumerate(tmpl):
                if len(group) > 1:
                    job = N.FactorJob.from_buffer_copy(t)
                    job.x.ptr = group[0][1][k]
                    table = N.segment_table([e[1][k] for e in group])
                    tables.append(table)
                    job.seg_ptrs, job.nseg = N.table_ptr(table), len(group)
                    if rag:
                        job.x.last_rows = group[-1][0][k].x.rows
                    jobs.append(job)
                else:
                    for i, e in enumerate(group):
                        job = N.FactorJob.from_buffer_copy(t)
                        job.x.ptr = e[1][k]
                        if i:
                            job.beta = 1.0  # later batches add to the first one's result
                        jobs.append(job)
            launches.append(jobs)
        # the groups of a flush (a pass's full batches and its short last one) as ONE
        # launch, each factor's jobs on their own accumulator slab ranges, when the
        # pending cycle's accumulators have a range for every job (or a new cycle
        # starts here); else one launch per group
        merged = [j for jobs in launches for j in jobs]
        if len(launches) > 1 and self.merge_launches and self._acc_takes(merged, device):
            launches = [merged]
        for jobs in launches:
            self._defer(jobs, device)
            N.factor_update(jobs, device)
        # queued records are released here (the host segment tables were read by the
        # calls); the caching allocator orders any reuse of the records' memory after
        # the launches on this stream
        del tables, queue

    @staticmethod
    def _ragged_ok(group, last, align):
        """`last` (one queued update) can be the ragged last batch of `group`'s
        multi-batch jobs: the same row-major factors, fewer rows, the per-batch-mean
        weighting (alpha x rows equal: the library weighs the last batch by
        rows / last_rows), the same operand alignment."""
        if align is not None and align[id(group[0])] != align[id(last)]:
            return False
        ta, tb = group[0][0], last[0]
        if len(ta) != len(tb):
            return False
        for a, b in zip(ta, tb):
            xa, xb = a.x, b.x
            if (xa.layout != N.ROWMAJOR or xb.layout != N.ROWMAJOR or xa.cols != xb.cols
                    or xa.has_ones != xb.has_ones or xa.ld != xb.ld or a.F != b.F
                    or xa.last_rows or xb.last_rows or not 0 < xb.rows < xa.rows):
                return False
            wa, wb = a.alpha * xa.rows, b.alpha * xb.rows
            if not abs(wa - wb) <= 1e-6 * abs(wa):
                return False
        return True

    def _acc_takes(self, jobs, device):
        """A launch of `jobs` fits the pending accumulation cycle: every factor it
        writes has an accumulator there, with a slab range per job of that factor."""
        if self._acc_map is None:
            return True
        if device != self._acc_device:
            return False
        count = {}
        for j in jobs:
            count[j.F] = count.get(j.F, 0) + 1
        return all(F in self._acc_map and n <= len(self._acc_map[F][1]) for F, n in count.items())

    def _defer(self, jobs, device):
        """Point each job at its factor's accumulator: continue the pending cycle when
        it holds a slab range for every job, else flush and plan a new cycle for this
        launch's jobs.  A factor written by k jobs of one launch gets k slab ranges of
        one accumulator (kfac_factor_job.acc_stride: the ranges' total; the flush sums
        them all); its i-th job in a launch takes the i-th range."""
        if self._acc_map is not None and not self._acc_takes(jobs, device):
            acc_jobs, self._acc_flush, self._acc_map = self._acc_flush, None, None
            self._end_cycle(acc_jobs)
        if self._acc_map is None:
            plan = N.factor_accum_plan(jobs)
            ranges, first = {}, {}
            for j, (splits, nbytes) in zip(jobs, plan):
                ranges.setdefault(j.F, []).append((splits, nbytes))
                first.setdefault(j.F, j)
            total, offs = 0, {}
            for F, rs in ranges.items():
                offs[F] = total
                total += sum(nb for _, nb in rs)  # (bytes are linear in the splits)
            buf = self._acc_buffer(total, device)
            base = buf.data_ptr()
            self._acc_map, self._acc_live, flush = {}, set(), []
            for F, rs in ranges.items():
                starts, s0 = [], 0
                for sp, _ in rs:
                    starts.append((s0, sp))
                    s0 += sp
                self._acc_map[F] = (base + offs[F], starts, s0)
                f = N.FactorJob.from_buffer_copy(first[F])
                f.seg_ptrs, f.nseg = None, 0
                f.acc, f.acc_splits, f.acc_stride = base + offs[F], s0, s0
                f.alpha = 1.0  # partials already carry alpha; f.beta: 0 fresh factor, 1 existing
                flush.append(f)
            self._acc_flush, self._acc_device = flush, device
        seen = {}
        for j in jobs:
            k = seen.get(j.F, 0)
            seen[j.F] = k + 1
            acc, starts, stride = self._acc_map[j.F]
            s0, sp = starts[k]
            j.acc, j.acc_splits, j.acc_stride = acc + s0 * _SLAB_BYTES, sp, stride
            j.acc_beta = 1.0 if (j.F, k) in self._acc_live else 0.0
            self._acc_live.add((j.F, k))

    def _acc_buffer(self, total, device):
        """The accumulator buffer of a new cycle (this turn's of the two), at least
        `total` bytes; the caller's stream first waits for a side-stream reduce still
        reading it (that wait also covers its release when it is regrown)."""
        par = self._acc_par
        buf = self._acc_bufs[par]
        if buf is not None:
            ev = self._acc_reads.pop(buf.data_ptr(), None)
            if ev is not None:
                if not ev.query():
                    ev.wait_on(N.stream_handle(buf.device))
                self._pool_event(buf.device, ev)
        if buf is None or buf.device != device or buf.numel() < total:
            buf = self._acc_bufs[par] = torch.empty(total, dtype=torch.uint8, device=device)
        return buf

    def _take_reduce(self):
        """For invert(): launch the queued updates and, when the pass's reduction is
        still deferred and can run on the inversion's side stream (reduce_on_side,
        overlap_invert, every factor of a latency-bound size), hand back its flush jobs
        instead of reducing on the caller's stream; else None (`state` reduces as usual)."""
        if not (self.reduce_on_side and self.overlap_invert and self.defer_reduce):
            return None
        if self._queue:
            self._launch_queue()
        self._launch_at = self.launch_first
        jobs = self._acc_flush
        if not jobs or not self._state or max(F_.shape[0] for v in self._state.values() for F_ in v) > 24 * 64:
            return None
        self._acc_flush = self._acc_map = None
        return jobs

    def _reduce_on_side(self, jobs, device, main_h, side_h):
        """The pass's deferred reduce on the side stream: after the caller's stream's
        launches, after the inversion that last read the target buffer; the event after
        it guards the accumulator buffer until the next cycle that takes it."""
        ev = self._event(device)
        ev.record(main_h)
        ev.wait_on(side_h)
        self._pool_event(device, ev)  # (the wait captured its record)
        self._await_readers(side_h)
        N.factor_flush(jobs, device, stream=side_h)
        done = self._event(device)
        done.record(side_h)
        buf = self._acc_bufs[self._acc_par]
        self._acc_reads[buf.data_ptr()] = done
        self._acc_par = (self._acc_par + 1) % len(self._acc_bufs)

    # ------------------------------------------------------------------ invert
    def _damping(self, add, multiply, count=None):
        """curvatures.py:373-378 argument handling, per state entry (`count`: the
        number of state entries, when the caller already holds them)."""
        if count is None:
            count = len(self.state)
        out = []
        for index in range(count):
            if not isinstance(add, (float, int)) and not isinstance(multiply, (float, int)):
                assert len(add) == len(multiply) == count
                n, s = add[index], multiply[index]
            else:
                n, s = float(add), float(multiply)
            out.append((n, s))
        return out

    def invert(self, add: Union[float, list, tuple] = 0., multiply: Union[float, list, tuple] = 1.):
        """L = cholesky(inverse(sqrt(s) F + sqrt(n) I)) per factor (curvatures.py:367-398)."""
        # the pass's deferred reduction: on the inversion's side stream (_take_reduce),
        # or completed here on the caller's stream by the `state` read
        side_reduce = self._take_reduce()
        handed = False  # the side stream has taken the pass's reduce
        try:
            state = self._state if side_reduce else self.state
            assert state, "State dict is empty. Did you call 'update' prior to this?"
            # a previous inversion's verdict (deferred mode) is settled or queued here
            self._defer_verdict()
            if self._inv_state:
                Warning("State has already been inverted. Is this expected?")
            entries = list(state.items())
            damping = self._damping(add, multiply, len(entries))
            for layer, (first, second) in entries:
                N.require_device(first, "state", layer)
                N.require_device(second, "state", layer)
            device = entries[0][1][0].device
            # The inversion runs on a high-priority side stream (overlap_invert): its
            # critical path is a chain of single-workgroup tile factorisations, so the
            # next data pass's SYRK launches fill the rest of the chip meanwhile.  The
            # side stream starts after the work that produced `state`; the caller's
            # stream waits only until the factors have been READ (kfac_invert_ex's
            # inputs_read event, after the first launch), so it may overwrite them.
            # Host side (round 4): one kfac_invert_pipelined call orders the side stream after
            # the caller's, runs the inversion, copies the verdict to pinned memory and
            # records `done`, on raw HIP events (N.RawEvent): ~10 torch.cuda stream / event
            # calls of 5-10 us each are gone from the caller's thread.  The L factors are
            # allocated on the caller's stream: every use or release of them is ordered after
            # `done` (_order_after), so the allocator's stream order covers the side stream.
            main_h = N.stream_handle(device)
            latency_bound = max(F_.shape[0] for _, v in entries for F_ in v) <= 24 * 64
            side = self._side_stream(device, alternate=latency_bound) if self.overlap_invert else None
            side_h = side.cuda_stream if side is not None else main_h
            outs, jobs = [], []
            for (layer, value), (n, s) in zip(entries, damping):
                pair = []
                for F_ in value:
                    out = torch.empty_like(F_, memory_format=torch.contiguous_format)
                    jobs.append(N.invert_job(F_, out, s ** 0.5, n ** 0.5))
                    pair.append(out)
                outs.append((layer, tuple(pair)))
            read = self._event(device) if side is not None else None
            done, order = self._event(device, ordering=False), self._event(device)
            host = self._pinned_host(len(jobs))
            after = main_h  # the stream the inversion is ordered after
            if side_reduce:
                if side is None or not latency_bound:  # (cannot happen: _take_reduce checked)
                    raise RuntimeError("KFAC.invert: side-stream reduce without a side stream")
                self._reduce_on_side(side_reduce, device, main_h, side_h)
                handed = True
                after = side_h
        except BaseException:
            # raised before the side stream took the reduce (validation, the previous
            # inversion's verdict, an allocation or event failure): reduce on the
            # caller's stream after all, so `state` never keeps unreduced factors
            if side_reduce and not handed:
                self._end_cycle(side_reduce)
            raise
        N.invert_pipelined(jobs, device, host, order, read, done, after, side_h, side)
        self._pool_event(device, order)  # (the side stream's wait captured its record)
        if read is not None:
            self._release(main_h, read, entries, device)
        for layer, pair in outs:
            self._inv_state[layer] = pair
        self._inv_pending = _Pending(done, host, [layer for layer, _ in outs], self._inv_state,
                                     [t for _, pair in outs for t in pair], side is not None)
        if self.eager_verdict:
            self._check_inverse()

    def _event(self, device, ordering=True):
        """A raw HIP event (N.RawEvent) from the pool of settled ones (a verdict's `done`
        after its host wait, an ordering event after the wait on it was enqueued).
        `ordering`: the event only orders streams on the device (no system-scope
        fence); a verdict's `done`, which the host waits on before reading the pinned
        copy, takes ordering=False."""
        ordering = ordering and _ORDERING_EVENTS
        pool = self._event_pool.get((device.index, ordering))
        return pool.pop() if pool else N.RawEvent(device, ordering=ordering)

    def _pool_event(self, device, ev):
        self._event_pool.setdefault((device.index, getattr(ev, "ordering", False)), []).append(ev)

    def _pinned_info(self, info):
        """A pinned host int32 buffer for a verdict readback (pooled)."""
        return self._pinned_host(info.numel())

    def _pinned_host(self, n):
        pool = self._info_pool
        while pool and pool[-1].numel() != n:
            pool.pop()
        return pool.pop() if pool else torch.empty(n, dtype=torch.int32, pin_memory=True)

    @staticmethod
    def _wait(ev, stream=None, device=None):
        """Order `stream`'s (default: the current stream's) later work after `ev`
        (a raw event or a torch.cuda.Event)."""
        if isinstance(ev, N.RawEvent):
            ev.wait_on(stream if isinstance(stream, int) else
                       stream.cuda_stream if stream is not None else N.stream_handle(device))
        else:
            (stream if stream is not None else torch.cuda.current_stream(device)).wait_event(ev)

    def _release(self, main_h, read, entries, device):
        """Let the caller's stream go past an inversion: straight away when the factors
        it reads are one of the double-buffered packed buffers (the buffer's next
        writer waits for `read` instead, see _await_readers), else behind `read`."""
        buf = self._packed
        if self.double_buffer and buf is not None:
            base = buf.untyped_storage().data_ptr()
            if all(F_.untyped_storage().data_ptr() == base for _, v in entries for F_ in v):
                self._buf_read[buf.data_ptr()] = read
                return
        read.wait_on(main_h)
        self._pool_event(device, read)

    def _side_stream(self, device, alternate=True):
        """The side stream of this inversion: two high-priority streams taken in turn,
        each with its own workspace (the library's workspace cache is per stream), so
        an inversion's F-reading launch does not queue behind the previous
        inversion's steps: the next data pass waits only for the factors to be read.
        A throughput-bound inversion (`alternate` False: some factor > 24 tiles of 64)
        always takes the first stream, so two of them never run at once and split the
        chip (wide MLP: 13.8 -> 25.5 ms per inversion when they did)."""
        s = self._inv_streams.get(device.index)
        if s is None:
            s = self._inv_streams[device.index] = _shared_side_streams(device)
        if not isinstance(s, list):  # a single stream set by hand (tools/probe_*.py)
            return s
        if not alternate:
            return s[0]
        self._inv_turn = getattr(self, "_inv_turn", 0) ^ 1
        return s[self._inv_turn]

    @classmethod
    def _order_after(cls, pending, settled=False):
        """Later work on the caller's stream sees the inversion's factors (no host wait).
        KFAC.invert allocates the factors on the caller's stream, so their release is
        ordered after this wait too; factors allocated on another stream (the sharded
        inversion's torch events) are also recorded on the caller's stream.  `settled`:
        the host has already waited for `done` (a raw event then needs no wait packet)."""
        if pending.on_side:
            dev = pending.outs[0].device
            if isinstance(pending.done, N.RawEvent):
                if not settled:
                    pending.done.wait_on(N.stream_handle(dev))
            else:
                cur = torch.cuda.current_stream(dev)
                cur.wait_event(pending.done)
                for t in pending.outs:
                    t.record_stream(cur)

    def _defer_verdict(self):
        """invert(): queue the pending inversion's verdict instead of waiting for it,
        and read the verdicts that are already back (at most `max_pending` stay queued).  Queued
        inversions are ordered before the caller's stream only when `inv_state` is
        read (_check_inverse), so the next data pass does not wait for them."""
        pending = getattr(self, "_inv_pending", None)
        if pending is not None:
            self._inv_pending = None
            self._inv_older.append(pending)
        while self._inv_older and (len(self._inv_older) > self.max_pending or self._inv_older[0].done.query()):
            p = self._inv_older.pop(0)
            # the verdict's host wait first (it settles `done`, also when it raises:
            # the factors are complete either way), then the stream order
            self._verdict(p)
            self._order_after(p, settled=True)

    def _check_inverse(self):
        """Settle every pending inversion, oldest first: a factor that is not positive
        definite ends as the reference's does (curvatures.py:393-396: torch fails, the
        numpy fallback raises LinAlgError), the layers from the first failing one on
        dropped from `inv_state` as the reference never assigns them."""
        older = getattr(self, "_inv_older", [])
        while older:
            p = older.pop(0)
            self._order_after(p)
            self._verdict(p)
        pending = getattr(self, "_inv_pending", None)
        if pending is None:
            return
        self._inv_pending = None
        self._order_after(pending)
        self._verdict(pending)

    def _verdict(self, pending):
        """Wait for one inversion's pivot check and act on it."""
        pending.done.synchronize()
        bad = pending.host.numpy().copy()
        self._info_pool.append(pending.host)
        if pending.outs and isinstance(pending.done, N.RawEvent):
            self._pool_event(pending.outs[0].device, pending.done)
        if bad.any():
            first = int(np.flatnonzero(bad)[0]) // 2  # two jobs (A, G) per layer
            for layer in pending.layers[first:]:
                pending.target.pop(layer, None)
            # the fp64 device factorisation fails exactly where numpy's fallback
            # would, so end the same way without a CPU path
            print("PyTorch Cholesky is singular. Using Numpy.")
            raise np.linalg.LinAlgError("Matrix is not positive definite")

    # ------------------------------------------------------------------ sample
    def sample(self, layer: Module) -> Tensor:
        """(L_A z L_G^T)^T, z ~ N(0, 1) (curvatures.py:400-405)."""
        assert self.inv_state, "Inverse state dict is empty. Did you call 'invert' prior to this?"
        first, second = self.inv_state[layer]
        z = torch.randn(first.size(0), second.size(0), device=first.device, dtype=first.dtype)
        first, second = first.contiguous(), second.contiguous()
        out = torch.empty(second.size(0), first.size(0), device=first.device, dtype=first.dtype)
        N.sample([N.sample_job(first, second, z, out, first.size(0))], first.device, accumulate=False)
        return out

    def sample_and_replace(self):
        """Curvature.sample_and_replace (curvatures.py:117-129) in one launch pair: the
        mean weights are restored, then every layer's (L_A z L_G^T)^T is added into its
        weight rows and bias (Curvature._replace, curvatures.py:68-82) by kfac_sample.
        z is drawn per layer in model.modules() order, as the reference draws it."""
        inv_state = self.inv_state
        assert inv_state, "Inverse state dict is empty. Did you call 'invert' prior to this?"
        self.model.load_state_dict(self.model_state)
        # the draws stay referenced until the launch is queued (a freed z would be
        # handed to the next draw by the caching allocator)
        jobs, draws, copies, device = [], [], [], None
        for layer in self.model.modules():
            if layer.__class__.__name__ not in self.layer_types:
                continue
            if layer.__class__.__name__ not in ['Linear', 'Conv2d']:
                continue
            first, second = inv_state[layer]
            nA, nG = first.size(0), second.size(0)
            z = torch.randn(nA, nG, device=first.device, dtype=first.dtype)
            # row-major factors (a column-major one, e.g. from torch.linalg.cholesky,
            # is copied; the copy is kept with the draws)
            first, second = first.contiguous(), second.contiguous()
            draws.extend((z, first, second))
            weight, bias = layer.weight.data, layer.bias.data if layer.bias is not None else None
            wcols = nA - 1 if bias is not None else nA
            if weight.numel() != nG * wcols:
                raise N.NativeError(f"sample_and_replace: {layer} weight has {weight.numel()} "
                                    f"elements, its factors give {nG} x {wcols}")
            target = weight
            if not weight.is_contiguous():
                # e.g. a channels_last Conv2d weight: the launch adds into a contiguous
                # copy, written back afterwards (the reference's _replace adds through
                # .contiguous().view(...) as well, curvatures.py:80-82)
                target = weight.contiguous()
                copies.append((weight, target))
            jobs.append(N.sample_job(first, second, z, target.view(nG, wcols), wcols, bias))
            device = first.device
        if jobs:
            N.sample(jobs, device, accumulate=True)
        for weight, target in copies:
            weight.copy_(target)


class EFB(Curvature):
    r"""Eigenvalue-corrected Kronecker factorisation (models/curvatures.py:408-470).

    The eigenbases of the KFAC factors come from the device eigensolver
    (`utilities.get_eigenvectors` -> kfac_syev; the reference's `torch.symeig` no longer
    exists on torch >= 2.0).  `update` projects each layer's batch gradient into the
    eigenbasis, lambda = (V_G^T grad V_A)^2 (two plain device GEMMs, rocBLAS via torch)
    and accumulates it; `sample` draws z * lambda^{-1/2} and maps it back through the
    eigenbases with kfac_sample (dense factors).
    """

    def __init__(self, model: Union[Module, Sequential], factors, layer_types: Union[List[str], str] = None):
        super().__init__(model, layer_types)
        from .utilities import get_eigenvectors
        self.eigvecs = get_eigenvectors(factors)
        self.diags = dict()

    def update(self, batch_size: int):
        """curvatures.py:427-449: state += (V_G^T grad V_A)^2, diags += grad^2 * B --
        every layer in one kfac_efb_update call (projection, square and accumulation
        fused; no lambdas tensor)."""
        # `keep`: the per-layer gradient matrices (torch.cat results) stay referenced
        # until the launch is queued -- a freed one could be handed by the caching
        # allocator to the next layer's tensors before the kernel reads it
        jobs, fresh, keep = [], [], []
        for layer in self.model.modules():
            if layer.__class__.__name__ in self.layer_types:
                if layer.__class__.__name__ in ['Linear', 'Conv2d']:
                    grads = layer.weight.grad.contiguous().view(layer.weight.grad.shape[0], -1)
                    if layer.bias is not None:
                        grads = torch.cat([grads, layer.bias.grad.unsqueeze(dim=1)], dim=1)
                    N.require_device(grads, "weight grad", layer)
                    V_A, V_G = self.eigvecs[layer]
                    if layer in self._state:
                        state, diag, accumulate = self._state[layer], self.diags[layer], True
                    else:
                        state = torch.empty_like(grads)
                        diag = torch.empty_like(grads)
                        accumulate = False
                        fresh.append((layer, state, diag))
                    jobs.append(N.efb_job(V_A, V_G, grads, state, diag, accumulate, batch_size))
                    keep.append(grads)
                elif layer.__class__.__name__ == 'MultiheadAttention':
                    raise NotImplementedError
        if jobs:
            N.efb_update(jobs, self._device_of(jobs))
        del keep
        for layer, state, diag in fresh:
            self._state[layer] = state
            self.diags[layer] = diag

    def _device_of(self, jobs):
        return next(iter(self.eigvecs.values()))[0].device

    def invert(self, add: Union[float, list, tuple] = 0., multiply: Union[float, list, tuple] = 1.):
        """curvatures.py:451-464: inv_state = (s * lambda + n)^{-1/2}, elementwise.  The
        reference tests `isinstance(.., float)` here (not int): an int damping is treated
        as a list and fails its length assert, as there."""
        assert self.state, "State dict is empty. Did you call 'update' prior to this?"
        if self.inv_state:
            Warning("State has already been inverted. Is this expected?")
        for index, (layer, value) in enumerate(self.state.items()):
            if not isinstance(add, float) and not isinstance(multiply, float):
                assert len(add) == len(multiply) == len(self.state)
                n, s = add[index], multiply[index]
            else:
                n, s = add, multiply
            self._inv_state[layer] = torch.reciprocal(s * value + n).sqrt()

    def sample(self, layer: Module) -> Tensor:
        """curvatures.py:466-473: (V_A (z * lambda^T) V_G^T)^T, z ~ N(0, 1)."""
        assert self.inv_state, "Inverse state dict is empty. Did you call 'invert' prior to this?"
        first, second = self.eigvecs[layer]
        lambdas = self.inv_state[layer]
        z = torch.randn(first.size(0), second.size(0), device=first.device, dtype=first.dtype)
        z *= lambdas.t()
        first, second = first.contiguous(), second.contiguous()
        out = torch.empty(second.size(0), first.size(0), device=first.device, dtype=first.dtype)
        N.sample([N.sample_job(first, second, z, out, first.size(0), dense=True)], first.device,
                 accumulate=False)
        return out


class INF(Curvature):
    r"""Low-rank EFB + diagonal correction (models/curvatures.py:476-682) on the device.

    `update(rank)` keeps the top-|lambda| eigenvector pairs (`_dim_reduction`, the
    reference's 1-based index arithmetic restated in tensor form) and the diagonal
    correction diag - sif_diag, where sif_diag (`_diagonal_accumulator`, a per-row loop
    over kron products in the reference) is ONE GEMM chain: (V_A*V_A) Lambda (V_G*V_G)^T.
    `invert` forms the pre-sample; V_s^T V_s is contracted without materialising the
    (nA*nG x r) kron(U_A, U_G) the reference builds (`pre_sampler`, :545-580).
    """

    def __init__(self, model: Union[Module, Sequential], diags, factors, lambdas,
                 layer_types: Union[List[str], str] = None):
        super().__init__(model, layer_types)
        assert diags.keys() == factors.keys() == lambdas.keys()
        from .utilities import get_eigenvectors
        self.eigvecs = get_eigenvectors(factors)
        self.lambdas = lambdas
        self.diags = diags

    def update(self, rank: int = 100):
        """curvatures.py:499-520."""
        for layer, (xxt_eigvecs, ggt_eigvecs), lambdas, diags in zip(
                list(self.diags.keys()), list(self.eigvecs.values()), list(self.lambdas.values()),
                list(self.diags.values())):
            N.require_device(lambdas, "lambdas", layer)
            lambda_vec = lambdas.t().contiguous().view(-1)
            diag_vec = diags.t().contiguous().view(-1)
            lr_a, lr_g, lr_lambda = self._dim_reduction(xxt_eigvecs, ggt_eigvecs, lambda_vec, rank)
            sif_diag = self._diagonal_accumulator(lr_a, lr_g, lr_lambda)
            self._state[layer] = (lr_a, lr_g, lr_lambda, diag_vec - sif_diag)

    def invert(self, add: Union[float, list, tuple] = 0., multiply: Union[float, list, tuple] = 1.):
        """curvatures.py:522-540 (float damping or lists, as the reference tests it)."""
        assert self.state, "State dict is empty. Did you call 'update' prior to this?"
        if self.inv_state:
            Warning("State has already been inverted. Is this expected?")
        for index, (layer, value) in enumerate(self.state.items()):
            if not isinstance(add, float) and not isinstance(multiply, float):
                assert len(add) == len(multiply) == len(self.state)
                n, s = add[index], multiply[index]
            else:
                n, s = add, multiply
            lr_a, lr_g, lr_lambda, correction = value
            correction[correction < 0] = 0
            reg_lr_lambda = (s * lr_lambda).sqrt()
            reg_inv_correction = torch.reciprocal(s * correction + n).sqrt()
            pre_sample = self.pre_sampler(lr_a, lr_g, reg_lr_lambda, reg_inv_correction)
            self._inv_state[layer] = (lr_a, lr_g, reg_inv_correction, pre_sample)

    def sample(self, layer: Module) -> Tensor:
        """curvatures.py:542-546."""
        assert self.inv_state, "Inverse state dict is empty. Did you call 'invert' prior to this?"
        a, b, c, d = self.inv_state[layer]
        return self.sampler(a, b, c, d).reshape(a.shape[0], b.shape[0]).t()

    @staticmethod
    def pre_sampler(frst_eigvecs: Tensor, scnd_eigvecs: Tensor, reg_lambda: Tensor,
                    reg_inv_correction: Tensor) -> Tensor:
        """curvatures.py:548-580.  V_s = c * kron(U_A, U_G) diag(sigma) is never formed:
        (V_s^T V_s)[(p,q),(p',q')] = sigma sigma' sum_a U_A[a,p] U_A[a,p'] T[a,q,q'],
        T[a] = U_G^T diag(c[a,:]^2) U_G -- two device GEMMs (kfac_kron_gram) whose
        operands are formed in the panel loaders."""
        vtv = N.kron_gram(frst_eigvecs, scnd_eigvecs, reg_inv_correction, reg_lambda)
        return INF._pre_sample_from_gram(vtv, reg_lambda)

    @staticmethod
    def _pre_sample_from_gram(vtv: Tensor, reg_lambda: Tensor, chol_inverse=None) -> Tensor:
        """curvatures.py:567-580 on the scaled Gram matrix.  The reference forms
        A = chol(vtv)^-1, B = chol(vtv + I), C = A^T (B - I) A and L_c = (C^-1 + vtv)^-1
        with two general inverses.  With vtv = L L^T, C^-1 = L (B - I)^-1 L^T, so
        C^-1 + vtv = L (B - I)^-1 B L^T and
            L_c = A^T (I - B^-1) A
        -- the same matrix from two triangular Cholesky inverses (kfac_invert on the
        device, fp64 inside: _chol_inverse) and two GEMMs, no general inverse.  On the
        reference's own G11 inputs it is 1e-12 from the fp64 literal chain and <= 8e-7
        with fp32 factors and GEMMs, where the reference's fp32 chain is up to 1.4e-4 off
        (cond(vtv) ~2e5 at full rank)."""
        vtv = (vtv + vtv.t()) / 2.
        eye = torch.eye(vtv.shape[0], device=vtv.device, dtype=vtv.dtype)
        A, B_inv = (chol_inverse or INF._chol_inverse)(vtv, (0.0, 1.0))
        L_c = A.t() @ (eye - B_inv) @ A
        return reg_lambda[:, None] * L_c * reg_lambda[None, :]

    @staticmethod
    def _chol_inverse(R: Tensor, shifts) -> list:
        """[chol(R + t I)^-1 for t in shifts] (lower) by ONE grouped kfac_invert: it
        computes X = chol(P R' P)^-1 and returns L = P X^T P (P the exchange matrix),
        so with R' = P R P (the flipped input) X = chol(R)^-1 = P L^T P."""
        N.require_device(R, "INF Gram matrix")
        Rf = torch.flip(R, (0, 1)).contiguous()
        outs = [torch.empty_like(Rf) for _ in shifts]
        info = N.invert([N.invert_job(Rf, o, 1.0, float(t)) for o, t in zip(outs, shifts)], R.device)
        if bool(info.any()):  # torch.linalg.cholesky's error in the reference
            raise RuntimeError("cholesky: The factorization could not be completed because the input "
                               "is not positive-definite.")
        return [torch.flip(o, (0, 1)).t() for o in outs]

    @staticmethod
    def sampler(frst_eigvecs: Tensor, scnd_eigvecs: Tensor, reg_inv_correction: Tensor,
                pre_sample: Tensor) -> Tensor:
        """curvatures.py:582-612."""
        X = torch.randn(frst_eigvecs.shape[0] * scnd_eigvecs.shape[0], device=frst_eigvecs.device,
                        dtype=frst_eigvecs.dtype)
        Y_l = reg_inv_correction * X
        unvec_Y_l = Y_l.reshape((scnd_eigvecs.shape[0], frst_eigvecs.shape[0]))
        Xq = scnd_eigvecs.t() @ unvec_Y_l @ frst_eigvecs
        Qx = pre_sample @ Xq.t().contiguous().view(-1)
        unvec_Qx = Qx.reshape((scnd_eigvecs.shape[1], frst_eigvecs.shape[1]))
        X_p_s = scnd_eigvecs @ unvec_Qx @ frst_eigvecs.t()
        Y_r = reg_inv_correction ** 2 * X_p_s.t().contiguous().view(-1)
        return Y_l - Y_r

    @staticmethod
    def _dim_reduction(frst_eigvecs: Tensor, scnd_eigvecs: Tensor, lambda_vec: Tensor, rank: int):
        """curvatures.py:614-660: the rows (a) and columns (g) of the top-`rank` |lambda|
        entries of the (nA x nG) lambda grid, each set unique and ascending, and the
        lambda sub-grid they span (row-major)."""
        if rank >= lambda_vec.shape[0]:
            return frst_eigvecs, scnd_eigvecs, lambda_vec
        m = scnd_eigvecs.shape[1]
        top = torch.argsort(-torch.abs(lambda_vec))[:rank]
        left = torch.unique(top // m)
        right = torch.unique(top % m)
        lr_lambda = lambda_vec.view(-1, m)[left][:, right].reshape(-1)
        return frst_eigvecs[:, left], scnd_eigvecs[:, right], lr_lambda

    @staticmethod
    def _diagonal_accumulator(xxt_eigvecs: Tensor, ggt_eigvecs: Tensor, lambda_vec: Tensor):
        """curvatures.py:662-682: diag[i*m + j] = sum_{p,q} U_A[i,p]^2 U_G[j,q]^2
        Lambda[p,q]; the reference's row loop over kron(U_A[i], U_G)^2 as one GEMM chain."""
        lam = lambda_vec.view(xxt_eigvecs.shape[1], ggt_eigvecs.shape[1])
        return ((xxt_eigvecs ** 2) @ lam @ (ggt_eigvecs ** 2).t()).reshape(-1)
