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
from abc import ABC, abstractmethod
from typing import Any, List, Union

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
        torch.save({'state': {names[k]: list(v) for k, v in self.state.items()},
                    'inv_state': {names[k]: list(v) for k, v in self.inv_state.items()},
                    'model': self.model.state_dict()}, filename)
        print('Writting %s complete!\n' % filename)

    def load(self, filename):
        blob = torch.load(filename, weights_only=True)
        modules = dict(self.model.named_modules())
        self.model.load_state_dict(blob['model'])
        self.state = {modules[k]: list(v) for k, v in blob['state'].items()}
        self.inv_state = {modules[k]: tuple(v) for k, v in blob['inv_state'].items()}
        print('Loading %s complete!\n' % filename)


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
                    # full hook: same grad_output[0] as the reference's legacy
                    # register_backward_hook for Linear/Conv2d (curvatures.py:315)
                    self.hooks.append(layer.register_full_backward_hook(self._save_output))
                elif layer.__class__.__name__ == 'MultiheadAttention':
                    raise NotImplementedError
        self._packed = None      # flat fp32 device buffer holding every factor
        self._packed_views = {}  # layer -> (A view, G view)
        self._layer_list = list(self.record)
        # Deferred reduction (kfac_factor_flush): updates keep each factor's split-K
        # partial tiles in device accumulators; the reduce into `state` runs once,
        # when the state is next read (invert / save / `state` / all-reduce).
        self.defer_reduce = True
        self._acc_buf = None     # grow-only device buffer of the accumulators
        self._acc_flush = None   # flush jobs of the pending cycle (None: nothing pending)
        self._acc_device = None

    def reset(self):
        """Forget the accumulated factors (start a new data pass); device buffers are kept."""
        self._acc_flush = None
        self._state = dict()
        self.inv_state = dict()

    def flush(self):
        """Reduce the pending accumulators into the factors (one launch; async)."""
        jobs = getattr(self, "_acc_flush", None)
        if jobs:
            self._acc_flush = None
            N.factor_flush(jobs, self._acc_device)

    # curvatures.py:319-323
    def _save_input(self, module, input):
        self.record[module][0] = input[0]

    def _save_output(self, module, grad_input, grad_output):
        self.record[module][1] = grad_output[0] * grad_output[0].size(0)

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
            x = forward.detach()
            if x.dim() != 4:
                raise RuntimeError(f"Conv2d KFAC expects a 4-D (B,C,H,W) input, got {tuple(x.shape)}")
            x = x.contiguous()
            g = backward.detach().contiguous()
            opA = N.patch_operand(x, layer.kernel_size, layer.padding, layer.stride, has_bias)
            opG = N.channel_operand(g)
            keep = (x, g)
        else:
            a = forward.detach()
            g = backward.detach()
            if a.dim() > 2 or g.dim() > 2:
                raise RuntimeError("t() expects a tensor with <= 2 dimensions, but self is "
                                   f"{max(a.dim(), g.dim())}D")
            a = a.reshape(1, -1) if a.dim() == 1 else a
            g = g.reshape(1, -1) if g.dim() == 1 else g
            if a.stride(-1) != 1:
                a = a.contiguous()
            if g.stride(-1) != 1:
                g = g.contiguous()
            opA = N.rowmajor_operand(a, has_bias)
            opG = N.rowmajor_operand(g, False)
            keep = (a, g)
        nA = opA.cols + opA.has_ones
        nG = opG.cols
        return opA, opG, nA, nG, keep

    def _alpha(self, op: N.Operand) -> float:
        """Per-batch mean: 1/cols (curvatures.py:349,356); an empty batch gives
        0 * inf = nan like the reference's 0/0."""
        return 1.0 / float(op.rows) if op.rows else float("inf")

    def _ensure_packed(self, sizes, device):
        """One flat buffer for all factors, views in modules() order."""
        total = sum(nA * nA + nG * nG for _, nA, nG in sizes)
        if self._packed is not None and self._packed.numel() == total and self._packed.device == device:
            return
        buf = torch.empty(total, dtype=torch.float32, device=device)
        views, off = {}, 0
        for layer, nA, nG in sizes:
            A = buf[off:off + nA * nA].view(nA, nA)
            off += nA * nA
            G = buf[off:off + nG * nG].view(nG, nG)
            off += nG * nG
            views[layer] = (A, G)
        self._packed, self._packed_views = buf, views

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
        jobs = []
        for layer, opA, opG, nA, nG, _keep in prepared:
            A, G, beta = self._target(layer, nA, nG, device)
            jobs.append(N.factor_job(opA, A, self._alpha(opA), beta))
            jobs.append(N.factor_job(opG, G, self._alpha(opG), beta))
        if self.defer_reduce:
            self._defer(jobs, device)
        N.factor_update(jobs, device)

    def _defer(self, jobs, device):
        """Point each job at its accumulator: continue the pending cycle when it
        targets the same factors, else (first update, or new targets) flush and plan
        a new cycle for this batch shape."""
        pending = self._acc_flush
        if pending is not None and (device != self._acc_device or len(pending) != len(jobs)
                                    or any(p.F != j.F for p, j in zip(pending, jobs))):
            self.flush()
            pending = None
        if pending is not None:
            for p, j in zip(pending, jobs):
                j.acc, j.acc_splits, j.acc_beta = p.acc, p.acc_splits, 1.0
            return
        plan = N.factor_accum_plan(jobs)
        offs, total = [], 0
        for _splits, nbytes in plan:
            offs.append(total)
            total += (nbytes + 255) // 256 * 256
        buf = self._acc_buf
        if buf is None or buf.device != device or buf.numel() < total:
            buf = self._acc_buf = torch.empty(total, dtype=torch.uint8, device=device)
        base = buf.data_ptr()
        flush = []
        for j, (splits, _nbytes), off in zip(jobs, plan, offs):
            j.acc, j.acc_splits, j.acc_beta = base + off, splits, 0.0
            f = N.FactorJob.from_buffer_copy(j)
            f.alpha = 1.0  # partials already carry alpha; f.beta: 0 fresh factor, 1 existing
            flush.append(f)
        self._acc_flush, self._acc_device = flush, device

    # ------------------------------------------------------------------ invert
    def _damping(self, add, multiply):
        """curvatures.py:373-378 argument handling, per state entry."""
        out = []
        for index in range(len(self.state)):
            if not isinstance(add, (float, int)) and not isinstance(multiply, (float, int)):
                assert len(add) == len(multiply) == len(self.state)
                n, s = add[index], multiply[index]
            else:
                n, s = float(add), float(multiply)
            out.append((n, s))
        return out

    def invert(self, add: Union[float, list, tuple] = 0., multiply: Union[float, list, tuple] = 1.):
        """L = cholesky(inverse(sqrt(s) F + sqrt(n) I)) per factor (curvatures.py:367-398)."""
        assert self.state, "State dict is empty. Did you call 'update' prior to this?"
        if self.inv_state:
            Warning("State has already been inverted. Is this expected?")
        damping = self._damping(add, multiply)
        jobs, outs = [], []
        device = None
        for (layer, value), (n, s) in zip(self.state.items(), damping):
            first, second = value
            pair = []
            for F_ in (first, second):
                N.require_device(F_, "state", layer)
                out = torch.empty_like(F_, memory_format=torch.contiguous_format)
                jobs.append(N.invert_job(F_, out, s ** 0.5, n ** 0.5))
                pair.append(out)
                device = F_.device
            outs.append((layer, tuple(pair)))
        info = N.invert(jobs, device)
        bad = info.cpu()
        if bool((bad != 0).any()):
            # The reference falls back to numpy (curvatures.py:393-396), which raises for
            # a factor that is not positive definite; the fp64 device factorisation fails
            # exactly there, so end the same way without a CPU path.
            print("PyTorch Cholesky is singular. Using Numpy.")
            raise np.linalg.LinAlgError("Matrix is not positive definite")
        for layer, pair in outs:
            self.inv_state[layer] = pair

    # ------------------------------------------------------------------ sample
    def sample(self, layer: Module) -> Tensor:
        """(L_A z L_G^T)^T, z ~ N(0, 1) (curvatures.py:400-405)."""
        assert self.inv_state, "Inverse state dict is empty. Did you call 'invert' prior to this?"
        first, second = self.inv_state[layer]
        z = torch.randn(first.size(0), second.size(0), device=first.device, dtype=first.dtype)
        return (first @ z @ second.t()).t()
