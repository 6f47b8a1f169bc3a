"""GPU parity of the paired-step inversion chain (KFAC_INV_PAIR=1: two elimination
steps per launch, invert_tiles.inc inv_pair / inv_build2) vs the fp64 oracle, for tile
counts of every parity (T - 1 even: pairs only; odd: a last single step without its
diagonal), grouped jobs of different T in one chain, the pivot verdict of a
non-positive-definite factor, and the KFAC MLP golden through the default API.

Criterion as tests/test_gpu_invert.py: rtol 1e-4 of cholesky(inverse(sqrt(s) F +
sqrt(n) I)) in fp64 (reference: models/curvatures.py:381-398).
"""
import numpy as np
import pytest
import torch

from oracle import kfac_oracle as O

pytestmark = pytest.mark.gpu


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def _spd(n, rng, cond=1e4):
    q, _ = np.linalg.qr(rng.standard_normal((n, n)))
    ev = np.logspace(0, np.log10(cond), n)
    return ((q * ev) @ q.T).astype(np.float32)


@pytest.fixture
def paired(monkeypatch):
    monkeypatch.setenv("KFAC_INV_PAIR", "1")
    yield
    monkeypatch.delenv("KFAC_INV_PAIR", raising=False)


# T = ceil(n / 32): 1, 2, 3, 4, 5, 7, 8, 25, 25, 48 (T - 1 odd and even)
@pytest.mark.parametrize("n", [7, 33, 65, 100, 129, 200, 256, 785, 800, 1536])
def test_paired_sizes_vs_fp64(hip_device, paired, n):
    from bnn_kfac_amd import _native as N
    rng = np.random.default_rng(100 + n)
    F = _spd(n, rng)
    Ft = _t(F, hip_device)
    L = torch.empty_like(Ft)
    info = N.invert([N.invert_job(Ft, L, 200 ** 0.5, 0.04 ** 0.5)], hip_device)
    assert int(info.cpu()[0]) == 0
    ref = O.invert_factor(F, 0.04, 200)
    got = L.cpu().numpy()
    np.testing.assert_allclose(got, ref, rtol=1e-4, atol=1e-7 * np.abs(ref).max())
    assert np.all(np.triu(got, 1) == 0)


def test_paired_grouped_jobs(hip_device, paired):
    """One chain over jobs whose pair counts and parities differ (the MLP's 785, 128,
    129, 10 and more), replayed twice (the second from the cached graph) with other
    damping (node parameters rewritten in place)."""
    from bnn_kfac_amd import _native as N
    rng = np.random.default_rng(7)
    sizes = (785, 128, 129, 10, 100, 33)
    mats = [_spd(n, rng, 1e3) for n in sizes]
    Fs = [_t(F, hip_device) for F in mats]
    for s, d in ((200.0, 0.04), (50.0, 0.5)):
        outs = [torch.empty_like(F) for F in Fs]
        info = N.invert([N.invert_job(F, o, s ** 0.5, d ** 0.5) for F, o in zip(Fs, outs)], hip_device)
        assert not info.cpu().any()
        for F, o in zip(mats, outs):
            ref = O.invert_factor(F, d, s)
            np.testing.assert_allclose(o.cpu().numpy(), ref, rtol=1e-4, atol=1e-7 * np.abs(ref).max())


@pytest.mark.parametrize("n,bad", [(100, 70), (785, 5), (785, 700), (65, 33)])
def test_paired_pivot_verdict(hip_device, paired, n, bad):
    """A factor that is not positive definite: the verdict names the first failing
    column as the single-step chain does (pivots checked in the critical tasks)."""
    from bnn_kfac_amd import _native as N
    rng = np.random.default_rng(n + bad)
    F = _spd(n, rng, 10.0)
    F[bad, bad] = -1e6  # (after the flip, column n-1-bad of the eliminated matrix)
    Ft = _t(F, hip_device)
    out = torch.empty_like(Ft)
    info_pair = int(N.invert([N.invert_job(Ft, out, 1.0, 0.0)], hip_device).cpu()[0])
    import os
    os.environ["KFAC_INV_PAIR"] = "0"
    try:
        info_one = int(N.invert([N.invert_job(Ft, out, 1.0, 0.0)], hip_device).cpu()[0])
    finally:
        os.environ["KFAC_INV_PAIR"] = "1"
    assert info_pair != 0
    assert info_pair == info_one


def test_paired_kfac_goldens(hip_device, paired):
    """The reference's own MLP / small-net inverses (G1 goldens) through KFAC.invert,
    with the paired chain: the same checks as tests/test_gpu_invert.py."""
    import test_gpu_invert as base
    base.test_kfac_invert_mlp_golden(hip_device)
    base.test_kfac_invert_small_golden(hip_device)
