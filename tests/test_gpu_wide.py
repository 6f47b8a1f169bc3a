"""GPU parity at the wide MLP's sizes (BASELINE C5: 784-4096-4096-10, factors 4097^2 and
4096^2), against the fp64 oracle:

* the SYRK of a 4096-wide layer (A 4097^2 with the ones column, G 4096^2) through
  KFAC.update (curvatures.py:345-363), rtol 1e-5 of the factor's scale;
* KFAC.invert at n = 4097 / 4096 (curvatures.py:381-398): the 64-tile two-launch
  path (inv_panel + inv_update, T = 65 tiles per edge), atol 1e-4 of max|L|
  (the north-star figure) vs cholesky(inv(R)) in fp64 on the device's own factor;
* eigenvalues at n = 4097 (utilities.py:120-141) vs LAPACK eigvalsh in fp64.
"""
import numpy as np
import pytest
import torch

from oracle import kfac_oracle as O

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def wide_layer(hip_device):
    """One update of a Linear(4096, 4096) layer over 1024 rows (U[0,1) inputs, N(0,1)
    gradient records), plus the fp64 truth of both factors."""
    from bnn_kfac_amd.curvatures import KFAC
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(4096, 4096)).to(hip_device)
    kfac = KFAC(net)
    rng = np.random.default_rng(4096)
    a = rng.random((1024, 4096), dtype=np.float32)
    g = rng.standard_normal((1024, 4096), dtype=np.float32)
    kfac.record[net[0]] = [torch.from_numpy(a).to(hip_device), torch.from_numpy(g).to(hip_device)]
    kfac.update(batch_size=1024)
    A, G = (t.cpu().numpy() for t in kfac.state[net[0]])
    wantA = O.linear_factor_A(a, True, np.float64)
    wantG = O.grad_factor(g, np.float64)
    return kfac, net, A, G, wantA, wantG


def test_wide_syrk_vs_fp64(wide_layer):
    _, _, A, G, wantA, wantG = wide_layer
    assert A.shape == (4097, 4097) and G.shape == (4096, 4096)
    for got, want in ((A, wantA), (G, wantG)):
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5 * np.abs(want).max())
        assert np.array_equal(got, got.T)  # written exactly symmetric


def test_wide_invert_4097_vs_fp64(wide_layer):
    kfac, net, A, G, _, _ = wide_layer
    kfac.invert(0.2 ** 2, 200)
    LA, LG = (t.cpu().numpy() for t in kfac.inv_state[net[0]])
    for L, F in ((LA, A), (LG, G)):
        want = O.invert_factor(F.astype(np.float64), 0.04, 200)
        np.testing.assert_allclose(L, want, rtol=0, atol=1e-4 * np.abs(want).max())
        assert np.all(np.triu(L, 1) == 0)


def test_wide_eigvals_4097(wide_layer, hip_device):
    from bnn_kfac_amd.utilities import symeig
    _, _, A, _, _, _ = wide_layer
    (ev, _), = symeig([torch.from_numpy(A).to(hip_device)])
    ev = ev.cpu().numpy()
    want = np.linalg.eigvalsh(A.astype(np.float64))
    assert ev.shape == (4097,) and np.all(np.diff(ev) >= 0)
    np.testing.assert_allclose(ev, want, rtol=1e-9, atol=1e-11 * np.abs(want).max())


def test_wide_queued_pass_vs_fp64(hip_device):
    """The C5 bench's launch shape: a Linear(4096, 4096) layer's updates QUEUED into one
    multi-batch kfac_factor_syrk3 launch (launch_first 16, the 512 MiB records cap: two
    4096-row batches per launch, as bench.py's wide pass runs them), then a shorter third
    batch (the ragged-tail path: its own launch on top), deferred reduction -- against
    the fp64 oracle's sum of per-batch means (curvatures.py:345-363), rtol 1e-5 of each
    factor's scale."""
    from bnn_kfac_amd.curvatures import KFAC
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(4096, 4096)).to(hip_device)
    kfac = KFAC(net)
    kfac.launch_first = 16
    rng = np.random.default_rng(40961)
    wantA = np.zeros((4097, 4097))
    wantG = np.zeros((4096, 4096))
    for rows in (4096, 4096, 1500):
        a = rng.random((rows, 4096), dtype=np.float32)
        g = rng.standard_normal((rows, 4096), dtype=np.float32)
        kfac.record[net[0]] = [torch.from_numpy(a).to(hip_device), torch.from_numpy(g).to(hip_device)]
        kfac.update(batch_size=rows)
        wantA += O.linear_factor_A(a, True, np.float64)
        wantG += O.grad_factor(g, np.float64)
    A, G = (t.cpu().numpy() for t in kfac.state[net[0]])
    for got, want in ((A, wantA), (G, wantG)):
        np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-5 * np.abs(want).max())
        assert np.array_equal(got, got.T)
