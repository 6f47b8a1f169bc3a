"""Data-parallel KFAC factor pass: one process per GPU, one all-reduce per pass.

The reference is single-device; its state is a SUM of per-batch means
(models/curvatures.py:359-363), i.e. linear in the per-batch contributions.  So a
global batch of B_global rows split over `world` ranks gives exactly the
reference's state when every rank accumulates

    sum_b (1 / B_global) * X_b,rank^T X_b,rank

locally (alpha = 1/B_global instead of 1/B_local) and the ranks' packed factor
buffers are summed ONCE after the pass (torch.distributed all_reduce; with the
"nccl" backend that is RCCL over xGMI).  Inversion is then replicated on every
rank (small factors) — no second collective.
"""
from __future__ import annotations

from typing import List, Union

import torch
import torch.distributed as dist
from torch.nn import Module, Sequential

from .curvatures import KFAC


class DistributedKFAC(KFAC):
    """KFAC whose update() consumes this rank's shard of each global batch.

    `update(batch_size, global_batch_size=None)`: the per-batch mean is taken over
    the GLOBAL batch (default: world_size x the local rows, i.e. equal shards).
    Local contributions accumulate into a private packed buffer; `allreduce()`
    (called by `invert()` if needed) sums it over ranks into `state`.
    """

    def __init__(self, model: Union[Module, Sequential], layer_types: Union[List[str], str] = None,
                 process_group=None):
        super().__init__(model, layer_types)
        self.group = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self._scale = 1.0          # local rows -> global rows for the current update
        self._local_state = {}     # rank-local accumulation (views of the packed buffer)
        self._pending = False
        self._global_buf, self._global_views = None, {}

    def _alpha(self, op) -> float:
        return 1.0 / (float(op.rows) * self._scale) if op.rows else float("inf")

    def update(self, batch_size: int, global_batch_size: int = None):
        if global_batch_size is None:
            self._scale = float(self.world)
        else:
            self._scale = float(global_batch_size) / float(batch_size)
        # accumulate into the rank-local state, then restore the reduced one (raw
        # dicts: reading `state` would complete the deferred reduction every update)
        reduced = self._state
        self._state = self._local_state
        try:
            super().update(batch_size)
        finally:
            self._local_state = self._state
            self._state = reduced
        self._pending = True

    def allreduce(self):
        """Sum the rank-local factors over ranks and add them to `state` (one collective)."""
        if not self._pending:
            return
        self.flush()  # the rank-local factors are complete only after the deferred reduce
        local = self._local_state
        packed = self._packed
        views_packed = packed is not None and all(
            local[layer][0].data_ptr() == self._packed_views[layer][0].data_ptr() for layer in local)
        if self.world > 1:
            if views_packed:
                dist.all_reduce(packed, op=dist.ReduceOp.SUM, group=self.group)
            else:
                for A, G in local.values():
                    dist.all_reduce(A, group=self.group)
                    dist.all_reduce(G, group=self.group)
        if not self._state:
            # first pass: the reduced local buffer becomes the state (no copy); the next
            # local accumulation gets a fresh buffer
            self._state = {layer: list(v) for layer, v in local.items()}
            self._global_buf, self._global_views = packed, self._packed_views
            self._packed = None
            self._packed_views = {}
        else:
            for layer, (A, G) in local.items():
                if layer in self._state:
                    self._state[layer][0] += A
                    self._state[layer][1] += G
                else:
                    self._state[layer] = [A.clone(), G.clone()]
        self._local_state = {}
        self._pending = False

    def invert(self, add=0., multiply=1.):
        self.allreduce()
        return super().invert(add, multiply)

    def reset(self):
        """Start a new pass, recycling the buffer the previous pass reduced into."""
        if self._global_buf is not None and self._packed is None:
            self._packed, self._packed_views = self._global_buf, self._global_views
            self._global_buf, self._global_views = None, {}
        super().reset()
        self._local_state = {}
        self._pending = False


def init_from_env(backend: str = None):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/MASTER_*)."""
    import os
    if dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world == 1:
        return 0, 1
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if backend == "nccl":
        torch.cuda.set_device(int(os.environ.get("LOCAL_RANK", "0")))
    dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()
