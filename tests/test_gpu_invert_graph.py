"""GPU: the inversion's hipGraph cache (invert_tiles.inc launch_steps_graph) gives the
same bits as the uncached per-step launches (KFAC_INV_GRAPH=0) of
models/curvatures.py:381-396's L = cholesky(inverse(sqrt(s)F + sqrt(n)I)):

* a damping grid over one shape (the cached graph's nodes re-parameterised in place);
* a call whose values differ from a replay that is still queued on the same stream
  (new damping AND new outputs, no host sync in between): the busy entry keeps its
  arguments and another entry is used;
* more distinct shapes than the cache holds (eviction waits for the last replay);
* kfac_release() mid-process (every cached graph destroyed, later calls rebuild).
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _spd(n, rng):
    X = rng.standard_normal((2 * n, n)).astype(np.float32)
    return (X.T @ X / (2 * n)).astype(np.float32)


def _invert(factors, damping, dev):
    """One grouped inversion on the current stream; returns (outs, info) unsynchronised."""
    from bnn_kfac_amd import _native as N
    outs = [torch.full_like(F, float("nan")) for F in factors]
    jobs = [N.invert_job(F, o, s ** 0.5, n ** 0.5) for F, o, (n, s) in zip(factors, outs, damping)]
    return outs, N.invert(jobs, dev)


def _uncached(factors, damping, dev):
    from bnn_kfac_amd import _native as N
    N.set_knob("KFAC_INV_GRAPH", 0)  # (the library reads its environment once, at load)
    try:
        outs, info = _invert(factors, damping, dev)
        torch.cuda.synchronize()
    finally:
        N.set_knob("KFAC_INV_GRAPH", 1)
    assert not info.any()
    return [o.cpu() for o in outs]


@pytest.fixture
def mlp_factors(hip_device):
    rng = np.random.default_rng(21)
    return [torch.from_numpy(_spd(n, rng)).to(hip_device) for n in (785, 128, 129, 10)]


def test_damping_grid_bit_exact(hip_device, mlp_factors):
    for add in (0.04, 1.0, 1e-3):
        for mult in (200.0, 1.0):
            d = [(add, mult)] * 4
            outs, info = _invert(mlp_factors, d, hip_device)
            torch.cuda.synchronize()
            assert not info.any()
            for got, want in zip(outs, _uncached(mlp_factors, d, hip_device)):
                assert torch.equal(got.cpu(), want)


def test_reparameterised_while_previous_replay_in_flight(hip_device, mlp_factors):
    d1, d2, d3 = [(0.04, 200.0)] * 4, [(1.0, 10.0)] * 4, [(0.3, 50.0)] * 4
    _invert(mlp_factors, d1, hip_device)  # builds (or refreshes) the cached graph
    torch.cuda.synchronize()
    # three calls back to back on one stream: the second and third change the values
    # of a graph whose replay is still queued / running
    o1, i1 = _invert(mlp_factors, d1, hip_device)
    o2, i2 = _invert(mlp_factors, d2, hip_device)
    o3, i3 = _invert(mlp_factors, d3, hip_device)
    torch.cuda.synchronize()
    for outs, info, d in ((o1, i1, d1), (o2, i2, d2), (o3, i3, d3)):
        assert not info.any()
        for got, want in zip(outs, _uncached(mlp_factors, d, hip_device)):
            assert torch.equal(got.cpu(), want)


def test_eviction_and_release(hip_device):
    from bnn_kfac_amd import _native as N
    rng = np.random.default_rng(5)
    shapes = [(n, n // 2 + 1) for n in (40, 70, 100, 130, 160, 190, 220, 250, 280, 310)]  # > 8 entries
    facs = {s: [torch.from_numpy(_spd(n, rng)).to(hip_device) for n in s] for s in shapes}
    d = [(0.04, 200.0)] * 2
    want = {s: _uncached(facs[s], d, hip_device) for s in shapes}
    for rep in range(2):
        pending = [(s,) + _invert(facs[s], d, hip_device) for s in shapes]  # no sync between
        torch.cuda.synchronize()
        for s, outs, info in pending:
            assert not info.any()
            for got, w in zip(outs, want[s]):
                assert torch.equal(got.cpu(), w)
        if rep == 0:
            assert N.lib().kfac_release() == 0  # every cached graph gone; the next calls rebuild
