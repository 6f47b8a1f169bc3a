"""GPU parity against fixtures made by the reference itself (tests/golden/make_goldens.py):

* G9 — KFAC hooks + update + invert on a net with nn.ReLU(inplace=True) after its
  Conv2d / Linear layers (curvatures.py:295-398).  Factors rtol 1e-5 (the device's
  backward rounds differently from the reference's CPU one: atol 1e-5 of the scale),
  L factors atol 1e-4 of max|L| vs the reference's fp32 L (its own error at this
  conditioning is below that).
* G10 — EFB (curvatures.py:408-473) on the reference's eigenbases and gradients:
  lambdas, diags, inverse, samples (the reference's draws injected).
* G11 — INF (curvatures.py:476-682): full rank through update/invert/sample; rank 6
  on the rows/columns the reference's index arithmetic selects.
* sample_and_replace on a channels_last Conv2d weight (non-contiguous).
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

from conftest import golden

pytestmark = pytest.mark.gpu


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def test_g9_inplace_relu_end_to_end(hip_device):
    from bnn_kfac_amd.curvatures import KFAC
    g = golden("g9_inplace.npz")
    net = nn.Sequential(nn.Conv2d(1, 4, 3, padding=1), nn.ReLU(inplace=True), nn.MaxPool2d(2),
                        nn.Flatten(), nn.Linear(64, 10), nn.ReLU(inplace=True), nn.Linear(10, 3))
    net.load_state_dict({k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("w_")})
    net = net.to(hip_device)
    kfac = KFAC(net)
    for bi in range(2):
        logits = net(_t(g[f"x{bi}"], hip_device))
        loss = nn.functional.cross_entropy(logits, _t(g[f"y{bi}"], hip_device))
        net.zero_grad()
        loss.backward()
        kfac.update(batch_size=8)
    kfac.invert(0.2 ** 2, 200)
    for li, layer in enumerate((net[0], net[4], net[6])):
        for got, key in zip(kfac.state[layer], ("A", "G")):
            want = g[f"{key}{li}"]
            np.testing.assert_allclose(got.cpu().numpy(), want, rtol=1e-5, atol=1e-5 * np.abs(want).max())
        for got, key in zip(kfac.inv_state[layer], ("LA", "LG")):
            want = g[f"{key}{li}"]
            np.testing.assert_allclose(got.cpu().numpy(), want, rtol=0, atol=1e-4 * np.abs(want).max())


def _efb_net(dev):
    torch.manual_seed(0)
    return nn.Sequential(nn.Conv2d(1, 3, 3), nn.ReLU(), nn.Flatten(), nn.Linear(3 * 4 * 4, 4)).to(dev)


def _golden_efb(dev):
    from bnn_kfac_amd.curvatures import EFB
    g = golden("g10_efb_inf.npz")
    net = _efb_net(dev)
    layers = [net[0], net[3]]
    factors = {m: [_t(g[f"A{i}"], dev), _t(g[f"G{i}"], dev)] for i, m in enumerate(layers)}
    efb = EFB(net, factors)
    efb.eigvecs = {m: (_t(g[f"VA{i}"], dev), _t(g[f"VG{i}"], dev)) for i, m in enumerate(layers)}
    for u in range(3):
        for i, m in enumerate(layers):
            m.weight.grad = _t(g[f"gw{u}_{i}"], dev)
            m.bias.grad = _t(g[f"gb{u}_{i}"], dev)
        efb.update(batch_size=32)
    return g, net, layers, factors, efb


def _inject_draws(monkeypatch, draws, dev):
    """torch.randn returns the reference's draws, in order (curvatures.py:469,594)."""
    queue = list(draws)

    def randn(*shape, device=None, dtype=None, **kw):
        z = queue.pop(0)
        assert tuple(z.shape) == tuple(shape if len(shape) != 1 or not isinstance(shape[0], tuple)
                                       else shape[0])
        return _t(z, dev)
    monkeypatch.setattr(torch, "randn", randn)


def test_g10_efb_vs_reference(hip_device, monkeypatch):
    g, net, layers, _, efb = _golden_efb(hip_device)
    for i, m in enumerate(layers):
        want = g[f"efb_lambda{i}"]
        np.testing.assert_allclose(efb.state[m].cpu().numpy(), want, rtol=1e-4, atol=1e-6 * want.max())
        np.testing.assert_allclose(efb.diags[m].cpu().numpy(), g[f"efb_diag{i}"], rtol=1e-5)
    efb.invert(0.04, 200.0)
    for i, m in enumerate(layers):
        np.testing.assert_allclose(efb.inv_state[m].cpu().numpy(), g[f"efb_inv{i}"], rtol=1e-4)
    _inject_draws(monkeypatch, [g["efb_z0"], g["efb_z1"]], hip_device)
    for i, m in enumerate(layers):
        want = g[f"efb_sample{i}"]
        np.testing.assert_allclose(efb.sample(m).cpu().numpy(), want, rtol=1e-4,
                                   atol=1e-4 * np.abs(want).max())


def test_g11_inf_full_rank_vs_reference(hip_device, monkeypatch):
    from bnn_kfac_amd.curvatures import INF
    g, net, layers, factors, efb = _golden_efb(hip_device)
    inf = INF(net, efb.diags, factors, efb.state)
    inf.eigvecs = efb.eigvecs
    inf.update(rank=10 ** 6)
    for i, m in enumerate(layers):
        a, b, lr, corr = (t.cpu().numpy() for t in inf.state[m])
        np.testing.assert_array_equal(a, g[f"inf_U_A{i}"])
        np.testing.assert_array_equal(b, g[f"inf_U_G{i}"])
        np.testing.assert_allclose(lr, g[f"inf_lr_lambda{i}"], rtol=1e-4, atol=1e-6 * lr.max())
        want = g[f"inf_correction{i}"]
        np.testing.assert_allclose(corr, want, rtol=1e-4, atol=1e-5 * np.abs(g[f"efb_diag{i}"]).max())
    inf.invert(0.04, 200.0)
    for i, m in enumerate(layers):
        c, P = (t.cpu().numpy() for t in inf.inv_state[m][2:])
        np.testing.assert_allclose(c, g[f"inf_reg_inv_correction{i}"], rtol=1e-3)
        want = g[f"inf_pre_sample{i}"]
        # V_s^T V_s is ill-conditioned at full rank: the reference's fp32 pre-sample is
        # ~5e-4 off the fp64 truth, the device's fp32 one likewise (normwise 2e-3)
        np.testing.assert_allclose(P, want, rtol=0, atol=2e-3 * np.abs(want).max())
    _inject_draws(monkeypatch, [g["inf_X0"], g["inf_X1"]], hip_device)
    for i, m in enumerate(layers):
        want = g[f"inf_sample{i}"]
        np.testing.assert_allclose(inf.sample(m).cpu().numpy(), want, rtol=0,
                                   atol=2e-3 * np.abs(want).max())


def test_g11_inf_rank6_vs_reference(hip_device, monkeypatch):
    from bnn_kfac_amd.curvatures import INF
    g, net, layers, factors, efb = _golden_efb(hip_device)
    inf = INF(net, efb.diags, factors, efb.state)
    inf.eigvecs = efb.eigvecs
    inf.update(rank=6)
    for i, m in enumerate(layers):
        a, b, lr, corr = (t.cpu().numpy() for t in inf.state[m])
        np.testing.assert_array_equal(a, g[f"VA{i}"][:, g[f"infr_left{i}"]])
        np.testing.assert_array_equal(b, g[f"VG{i}"][:, g[f"infr_right{i}"]])
        np.testing.assert_allclose(lr, g[f"infr_lr_lambda{i}"], rtol=1e-4)
        np.testing.assert_allclose(corr, g[f"infr_correction{i}"], rtol=1e-4,
                                   atol=1e-5 * np.abs(g[f"efb_diag{i}"]).max())
    inf.invert(0.04, 200.0)
    for i, m in enumerate(layers):
        c, P = (t.cpu().numpy() for t in inf.inv_state[m][2:])
        np.testing.assert_allclose(c, g[f"infr_reg_inv_correction{i}"], rtol=1e-3)
        want = g[f"infr_pre_sample{i}"]
        np.testing.assert_allclose(P, want, rtol=0, atol=1e-3 * np.abs(want).max())
    _inject_draws(monkeypatch, [g["infr_X0"], g["infr_X1"]], hip_device)
    for i, m in enumerate(layers):
        want = g[f"infr_sample{i}"]
        np.testing.assert_allclose(inf.sample(m).cpu().numpy(), want, rtol=0,
                                   atol=1e-3 * np.abs(want).max())


def test_sample_and_replace_channels_last(hip_device):
    """A channels_last Conv2d weight (non-contiguous) gets the same sample as a
    contiguous one (Curvature._replace adds through .contiguous().view, :80-82)."""
    from bnn_kfac_amd.curvatures import KFAC
    nets, kfacs = [], []
    for fmt in (torch.contiguous_format, torch.channels_last):
        torch.manual_seed(0)
        net = nn.Sequential(nn.Conv2d(3, 8, 3), nn.Flatten(), nn.Linear(8 * 4 * 4, 5)).to(hip_device)
        nets.append(net.to(memory_format=fmt))
        kfacs.append(KFAC(nets[-1]))
    x = torch.rand(16, 3, 6, 6, device=hip_device)
    nets[0](x).sum().backward()
    kfacs[0].update(16)
    kfacs[0].invert(0.04, 200)
    # the same inverse factors for both (the channels_last net's own forward/backward
    # would round differently): only the weight layout differs
    kfacs[1].inv_state = {m1: kfacs[0].inv_state[m0] for m0, m1 in
                          ((nets[0][0], nets[1][0]), (nets[0][2], nets[1][2]))}
    outs = []
    for net, kfac in zip(nets, kfacs):
        torch.manual_seed(3)
        kfac.sample_and_replace()
        outs.append([p.detach().contiguous().cpu().numpy() for p in net.parameters()])
    assert not nets[1][0].weight.is_contiguous()
    for a, b in zip(*outs):
        np.testing.assert_array_equal(a, b)
