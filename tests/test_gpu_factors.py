"""GPU parity: factor accumulation (KFAC.update) through libkfac_hip vs the oracle.

Tolerances: factors are fp32 sums of products; the kernel's fp32 MFMA chain and the
reference's MKL sgemm each sit ~1e-7 relative from the fp64 truth, so the
criterion is rtol 1e-5 against the fp64 oracle and the goldens.
"""
import numpy as np
import pytest
import torch
import torch.nn as nn

from conftest import golden
from oracle import kfac_oracle as O

pytestmark = pytest.mark.gpu

FT = dict(rtol=1e-5, atol=1e-6)


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


def test_mfma_layout_asymmetric(hip_device):
    """Raw C-ABI, one asymmetric operand: catches row/col swaps in the MFMA C-layout."""
    from bnn_kfac_amd import _native as N
    rng = np.random.default_rng(0)
    for B, d, ones in [(33, 70, True), (1, 1, False), (64, 64, True), (97, 129, False), (300, 10, True)]:
        x = rng.integers(-3, 4, size=(B, d)).astype(np.float32)  # exact small integers
        F = torch.full((d + ones, d + ones), np.nan, device=hip_device)
        N.factor_update([N.factor_job(N.rowmajor_operand(_t(x, hip_device), ones), F, 1.0, 0.0)],
                        hip_device)
        xo = np.concatenate([x, np.ones((B, 1), np.float32)], 1) if ones else x
        np.testing.assert_array_equal(F.cpu().numpy(), xo.T.astype(np.float64) @ xo)


def test_strided_rows_and_beta(hip_device):
    from bnn_kfac_amd import _native as N
    rng = np.random.default_rng(1)
    base = rng.standard_normal((200, 96)).astype(np.float32)
    xt = _t(base, hip_device)[:, 5:85]  # ld 96, cols 80
    F0 = rng.standard_normal((81, 81)).astype(np.float32)
    F0 = F0 + F0.T
    F = _t(F0, hip_device)
    N.factor_update([N.factor_job(N.rowmajor_operand(xt, True), F, 0.25, 1.0)], hip_device)
    x = base[:, 5:85].astype(np.float64)
    xo = np.concatenate([x, np.ones((200, 1))], 1)
    want = F0 + 0.25 * xo.T @ xo
    # F0 + x^T x cancels to near zero in places: absolute tolerance at the sum's scale
    np.testing.assert_allclose(F.cpu().numpy(), want, rtol=1e-5, atol=1e-6 * np.abs(0.25 * xo.T @ xo).max())


def test_small_linear_golden(hip_device):
    from bnn_kfac_amd.curvatures import KFAC
    g = golden("g1_small_linear.npz")
    net = nn.Sequential(nn.Linear(20, 12), nn.ReLU(), nn.Linear(12, 5, bias=False)).to(hip_device)
    kfac = KFAC(net)
    for bi in range(3):
        kfac.record[net[0]] = [_t(g[f"b{bi}_a1"], hip_device), _t(g[f"b{bi}_g1"], hip_device)]
        kfac.record[net[2]] = [_t(g[f"b{bi}_a2"], hip_device), _t(g[f"b{bi}_g2"], hip_device)]
        kfac.update(batch_size=len(g[f"b{bi}_a1"]))
    assert list(kfac.state.keys()) == [net[0], net[2]]
    for li, layer in enumerate([net[0], net[2]]):
        A, G = kfac.state[layer]
        np.testing.assert_allclose(A.cpu().numpy(), g[f"A{li}"], **FT)
        np.testing.assert_allclose(G.cpu().numpy(), g[f"G{li}"], **FT)
        assert torch.equal(A, A.t()) and torch.equal(G, G.t())


def mlp_batches(seed=123, sizes=(256, 256, 256, 96)):
    rng = np.random.default_rng(seed)
    for B in sizes:
        yield (B, rng.random((B, 784), dtype=np.float32), rng.standard_normal((B, 128), dtype=np.float32),
               rng.random((B, 128), dtype=np.float32), rng.standard_normal((B, 10), dtype=np.float32))


def test_mlp_golden_and_oracle(hip_device):
    from bnn_kfac_amd.curvatures import KFAC
    g = golden("g1_mlp.npz")
    net = nn.Sequential(nn.Linear(784, 128), nn.ReLU(), nn.Linear(128, 10)).to(hip_device)
    kfac = KFAC(net)
    ref = O.OracleKFAC(np.float64)
    for B, a1, g1, a2, g2 in mlp_batches():
        kfac.record[net[0]] = [_t(a1, hip_device), _t(g1, hip_device)]
        kfac.record[net[2]] = [_t(a2, hip_device), _t(g2, hip_device)]
        kfac.update(batch_size=B)
        ref.update_linear("fc1", a1, g1, True)
        ref.update_linear("fc2", a2, g2, True)
    A1, G1 = [t.cpu().numpy() for t in kfac.state[net[0]]]
    A2, G2 = [t.cpu().numpy() for t in kfac.state[net[2]]]
    np.testing.assert_allclose(A1, ref.state["fc1"][0], **FT)
    np.testing.assert_allclose(G1, ref.state["fc1"][1], **FT)
    np.testing.assert_allclose(A2, ref.state["fc2"][0], **FT)
    np.testing.assert_allclose(G2, ref.state["fc2"][1], **FT)
    np.testing.assert_allclose(np.diag(A1), g["A1_diag"], **FT)
    np.testing.assert_allclose(A1[:8], g["A1_head"], **FT)
    np.testing.assert_allclose(A1[-8:], g["A1_tail"], **FT)
    np.testing.assert_allclose(G1, g["G1"], **FT)
    np.testing.assert_allclose(A2, g["A2"], **FT)
    np.testing.assert_allclose(G2, g["G2"], **FT)


def test_conv_golden(hip_device):
    from bnn_kfac_amd.curvatures import KFAC
    g = golden("g4_conv.npz")
    convs = []
    for li in range(4):
        kh, kw, sh, sw, ph, pw, bias, cout = [int(v) for v in g[f"meta{li}"]]
        cin = g[f"x{li}"].shape[1]
        convs.append(nn.Conv2d(cin, cout, (kh, kw), stride=(sh, sw), padding=(ph, pw), bias=bool(bias)))
    net = nn.Sequential(*convs).to(hip_device)
    kfac = KFAC(net)
    for _ in range(2):
        for li, layer in enumerate(convs):
            kfac.record[layer] = [_t(g[f"x{li}"], hip_device), _t(g[f"g{li}"], hip_device)]
        kfac.update(batch_size=0)
    for li, layer in enumerate(convs):
        A, G = kfac.state[layer]
        np.testing.assert_allclose(A.cpu().numpy(), g[f"A{li}"], **FT)
        np.testing.assert_allclose(G.cpu().numpy(), g[f"G{li}"], **FT)


X3F_SPECS = [(16, 6, 14, 14, 16, (5, 5), (1, 1), (0, 0), True), (64, 6, 14, 14, 16, (5, 5), (1, 1), (0, 0), True),
             (3, 9, 5, 13, 5, (3, 4), (1, 1), (1, 2), True), (2, 10, 7, 8, 3, (3, 5), (1, 1), (1, 1), False),
             (3, 4, 10, 11, 4, (6, 6), (1, 1), (1, 1), True)]
X3S_SPECS = [(16, 1, 28, 28, 6, (5, 5), (1, 1), (2, 2), True), (256, 1, 28, 28, 6, (5, 5), (1, 1), (2, 2), True),
             (5, 2, 11, 13, 4, (3, 4), (2, 1), (1, 2), True),
             (3, 3, 12, 16, 5, (3, 3), (1, 1), (0, 1), False), (2, 2, 9, 9, 3, (4, 4), (1, 1), (1, 1), False)]


@pytest.mark.parametrize("spec", [
    # (B, Cin, H, W, Cout, k, stride, pad, bias): LeNet-5 / BaseNet_15k shapes + odd ones
    (16, 1, 28, 28, 6, (5, 5), (1, 1), (2, 2), True),
    (16, 6, 14, 14, 16, (5, 5), (1, 1), (0, 0), True),
    (8, 5, 12, 12, 10, (5, 5), (1, 1), (0, 0), True),
    (3, 7, 9, 11, 70, (3, 2), (2, 3), (1, 0), False),
    (2, 13, 6, 6, 3, (1, 1), (1, 1), (0, 0), True),
    # LDS-staged conv kernel: K splits inside images (B=64 / 256), 16x16 narrow im2col
    # factor (n=10) with a 32-wide channel factor, 1x1 outputs (positions wrap every
    # step), an im2col image too large to stage (register-staged fallback) next to a
    # staged 8000-float gradient block, and a channel block not float4-sized (fallback)
    (64, 6, 14, 14, 16, (5, 5), (1, 1), (0, 0), True),
    (256, 1, 28, 28, 6, (5, 5), (1, 1), (2, 2), True),
    (4, 1, 10, 10, 20, (3, 3), (1, 1), (1, 1), True),
    (6, 3, 5, 5, 4, (5, 5), (1, 1), (0, 0), True),
    (2, 3, 40, 40, 5, (3, 3), (1, 1), (1, 1), True),
    (2, 2, 5, 5, 3, (3, 3), (1, 1), (0, 0), True),
    # kfac_factor_conv_x3 (im2col factors with 32 < n <= 192, bf16x3 from an LDS
    # im2col): an image whose 1,024 positions take many LDS chunks, stride 2 without
    # bias, 33 and 181 features (2 / 6 blocks per edge: 1 / 3 blocks per wave, the latter
    # in 2 chunks of 32 positions), and 224 features (the fp32 kernel again)
    (4, 2, 32, 32, 6, (5, 5), (1, 1), (2, 2), True),
    (5, 4, 15, 15, 8, (3, 3), (2, 2), (1, 1), False),
    (3, 1, 20, 20, 4, (4, 8), (1, 1), (0, 0), True),
    (2, 20, 10, 10, 5, (3, 3), (1, 1), (0, 0), True),
    (2, 14, 9, 9, 6, (4, 4), (1, 1), (0, 0), False),
    # kfac_factor_conv_x3s (im2col factors with 17 <= n <= 32, bf16x3 from column-
    # shifted image copies; LeNet-5's conv1 above; 19 features over 3 groups above: an
    # odd group count, which stays on the fp32 kernel): row stride 2 with asymmetric
    # padding and 14 output columns (two groups per row, the second 6 wide), 27
    # features without bias over 16 columns (column stride 3: the fp32 kernel), n = 32
    (5, 2, 11, 13, 4, (3, 4), (2, 1), (1, 2), True),
    (3, 3, 12, 16, 5, (3, 3), (1, 1), (0, 1), False),
    (3, 3, 12, 17, 5, (3, 3), (1, 3), (0, 1), False),
    (2, 2, 9, 9, 3, (4, 4), (1, 1), (1, 1), False),
    # kfac_factor_conv_x3f (stride-1 im2col factors with 97 <= n <= 160 from flattened
    # column copies; LeNet-5's conv2 above): 4 block rows with two shifted variants (14
    # output columns, 70 positions: a masked last k-step), 5 block rows without bias
    # (two variants, 42 positions), 5 block rows with bias and a 6 x 6 kernel (one
    # variant, 56 positions)
    (3, 9, 5, 13, 5, (3, 4), (1, 1), (1, 2), True),
    (2, 10, 7, 8, 3, (3, 5), (1, 1), (1, 1), False),
    (3, 4, 10, 11, 4, (6, 6), (1, 1), (1, 1), True),
])
def test_conv_shapes_vs_oracle(hip_device, spec):
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import KFAC
    B, Cin, H, W, Cout, k, s, p, bias = spec
    rng = np.random.default_rng(sum(spec[:5]))
    conv = nn.Conv2d(Cin, Cout, k, stride=s, padding=p, bias=bias).to(hip_device)
    x = rng.random((B, Cin, H, W), dtype=np.float32)
    Ho, Wo = (H + 2 * p[0] - k[0]) // s[0] + 1, (W + 2 * p[1] - k[1]) // s[1] + 1
    gr = rng.standard_normal((B, Cout, Ho, Wo), dtype=np.float32)
    kfac = KFAC(conv)
    kfac.record[conv] = [_t(x, hip_device), _t(gr, hip_device)]
    N.profile_reset()
    N.profile_enable(True)
    kfac.update(batch_size=B)
    torch.cuda.synchronize()
    N.profile_enable(False)
    if spec in X3S_SPECS:  # the A factor on the column-copy kernel, one launch
        assert N.profile_read(N.PROF_FACTOR_CONV_X3S)[1] == 1
    if spec in X3F_SPECS:  # on the flattened column-copy kernel
        assert N.profile_read(N.PROF_FACTOR_CONV_X3F)[1] == 1
    A, G = kfac.state[conv]
    np.testing.assert_allclose(A.cpu().numpy(), O.conv_factor_A(x, k, p, s, bias, np.float64), **FT)
    np.testing.assert_allclose(G.cpu().numpy(), O.grad_factor(gr, np.float64), **FT)


@pytest.mark.gpu
@pytest.mark.parametrize("B,cout,hw", [(9000, 16, 10), (300, 11, 14), (40, 32, 6), (5, 9, 22)])
def test_channel_x3(hip_device, B, cout, hw):
    """G of a conv layer with 8 < n <= 32 on kfac_factor_channel_x3 (bf16x3 fragments
    straight from HBM, one diagonal block in four MFMAs): LeNet-5's conv2 G over 9,000
    images in one launch, and n = 11 / 32 / 9 over 196, 36 and 484 positions (a last
    k-step with 4 positions: half a float4 pair), fewer images than waves."""
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import KFAC
    rng = np.random.default_rng(B + cout)
    conv = nn.Conv2d(3, cout, 3, bias=True).to(hip_device)
    x = rng.random((B, 3, hw + 2, hw + 2), dtype=np.float32)
    gr = rng.standard_normal((B, cout, hw, hw), dtype=np.float32)
    kfac = KFAC(conv)
    kfac.record[conv] = [_t(x, hip_device), _t(gr, hip_device)]
    N.profile_reset()
    N.profile_enable(True)
    kfac.update(batch_size=B)
    torch.cuda.synchronize()
    N.profile_enable(False)
    assert N.profile_read(N.PROF_FACTOR_CHANNEL_X3)[1] == 1
    _, G = kfac.state[conv]
    np.testing.assert_allclose(G.cpu().numpy(), O.grad_factor(gr, np.float64), **FT)


@pytest.mark.gpu
@pytest.mark.parametrize("cout", [6, 16])
def test_channel_operand_with_ones(hip_device, cout):
    """A CHANNEL operand with a ones column (legal in the C ABI, unused by the hooks):
    F = [G | 1]^T [G | 1] on the unstaged kernel (the channel kernels have no ones row)."""
    from bnn_kfac_amd import _native as N
    B, L = 64, 36
    rng = np.random.default_rng(cout)
    g = rng.standard_normal((B, cout, L), dtype=np.float32)
    op = N.channel_operand(_t(g.reshape(B, cout, 6, 6), hip_device))
    op.has_ones = 1
    n = cout + 1
    F = torch.zeros((n, n), device=hip_device)
    N.factor_update([N.factor_job(op, F, 1.0, 0.0)], hip_device)
    torch.cuda.synchronize()
    X = np.concatenate([g.transpose(0, 2, 1).reshape(-1, cout), np.ones((B * L, 1), np.float32)], 1)
    W = X.T.astype(np.float64) @ X
    # (fp32 sums of 2,304 products on the fp32 kernel: entries near zero carry the
    # rounding of the whole sum, so the absolute bound is relative to max |W|)
    np.testing.assert_allclose(F.cpu().numpy(), W, rtol=1e-5, atol=1e-6 * np.abs(W).max())


@pytest.mark.gpu
@pytest.mark.parametrize("cout", [6, 7])
def test_channel_small_large_launch(hip_device, cout):
    """G of a conv layer over 9,000 images in one launch (the n <= 8 register-triangle
    kernel at 4 workgroups per CU past 8,192 images; 7: the n = 8 instance with a zero
    row)."""
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import KFAC
    B, Ho, Wo = 9000, 10, 10
    rng = np.random.default_rng(cout)
    conv = nn.Conv2d(3, cout, 3, bias=True).to(hip_device)
    x = rng.random((B, 3, Ho + 2, Wo + 2), dtype=np.float32)
    gr = rng.standard_normal((B, cout, Ho, Wo), dtype=np.float32)
    kfac = KFAC(conv)
    kfac.record[conv] = [_t(x, hip_device), _t(gr, hip_device)]
    N.profile_reset()
    N.profile_enable(True)
    kfac.update(batch_size=B)
    torch.cuda.synchronize()
    N.profile_enable(False)
    assert N.profile_read(N.PROF_FACTOR_CHANNEL_SMALL)[1] == 1
    _, G = kfac.state[conv]
    np.testing.assert_allclose(G.cpu().numpy(), O.grad_factor(gr, np.float64), **FT)


def test_hooks_end_to_end_basenet750(hip_device):
    """Full forward/backward through the hooks reproduces the reference's factors (G5)."""
    from bnn_kfac_amd.curvatures import KFAC
    from models_for_tests import BaseNet750
    g = golden("g5_basenet750.npz")
    net = BaseNet750()
    net.load_state_dict({k[2:]: torch.from_numpy(v) for k, v in g.items() if k.startswith("w_")})
    net = net.to(hip_device)
    kfac = KFAC(net)
    crit = nn.CrossEntropyLoss()
    for bi in range(2):
        x = _t(g[f"x{bi}"], hip_device)
        y = torch.from_numpy(g[f"y{bi}"]).to(hip_device)
        loss = crit(net(x), y)
        net.zero_grad()
        loss.backward()
        kfac.update(batch_size=8)
    for li, layer in enumerate([net.conv1, net.conv2, net.fc1]):
        A, G = kfac.state[layer]
        np.testing.assert_allclose(A.cpu().numpy(), g[f"A{li}"], rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(G.cpu().numpy(), g[f"G{li}"], rtol=1e-4, atol=1e-6)


def test_deterministic_and_large_batch(hip_device):
    """Bitwise-reproducible (no atomics) and right at B = 4096 (the bench shape)."""
    from bnn_kfac_amd.curvatures import KFAC
    torch.manual_seed(0)
    net = nn.Sequential(nn.Linear(784, 128), nn.ReLU(), nn.Linear(128, 10)).to(hip_device)
    a1 = torch.rand(4096, 784, device=hip_device)
    g1 = torch.randn(4096, 128, device=hip_device)
    outs = []
    for _ in range(2):
        kfac = KFAC(net)
        kfac.record[net[0]] = [a1, g1]
        kfac.record[net[2]] = [a1[:, :128], g1[:, :10]]
        kfac.update(4096)
        outs.append([t.clone() for t in kfac.state[net[0]]])
    assert torch.equal(outs[0][0], outs[1][0]) and torch.equal(outs[0][1], outs[1][1])
    ref = O.linear_factor_A(a1.cpu().numpy(), True, np.float64)
    np.testing.assert_allclose(outs[0][0].cpu().numpy(), ref, **FT)


def test_empty_batch_rows(hip_device):
    """A zero-row operand contributes exactly nothing and reads nothing."""
    from bnn_kfac_amd import _native as N
    x = torch.empty(0, 5, device=hip_device)
    F = torch.zeros(6, 6, device=hip_device)
    N.factor_update([N.factor_job(N.rowmajor_operand(x, True), F, 1.0, 1.0)], hip_device)
    assert torch.equal(F, torch.zeros_like(F))


def test_deferred_reduce_raw_abi(hip_device):
    """kfac_factor_update with accumulators + kfac_factor_flush: F0 + sum of three
    batches (the last one much smaller than the planned one, so trailing splits are
    empty), exact on small integers; F stays untouched until the flush."""
    from bnn_kfac_amd import _native as N
    rng = np.random.default_rng(5)
    F0 = rng.integers(-4, 5, size=(130, 130)).astype(np.float32)
    F0 = F0 + F0.T
    F = _t(F0, hip_device)
    xs = [rng.integers(-3, 4, size=(B, 129)).astype(np.float32) for B in (3000, 3000, 70)]
    xd = [_t(x, hip_device) for x in xs]
    jobs = [N.factor_job(N.rowmajor_operand(xd[0], True), F, 1.0, 1.0)]
    (splits, nbytes), = N.factor_accum_plan(jobs)
    assert splits >= 2
    acc = torch.empty(nbytes, dtype=torch.uint8, device=hip_device)
    for i, x in enumerate(xd):
        j = N.factor_job(N.rowmajor_operand(x, True), F, 1.0, 1.0)
        j.acc, j.acc_splits, j.acc_beta = acc.data_ptr(), splits, 0.0 if i == 0 else 1.0
        N.factor_update([j], hip_device)
    np.testing.assert_array_equal(F.cpu().numpy(), F0)
    f = N.factor_job(N.rowmajor_operand(xd[0], True), F, 1.0, 1.0)
    f.acc, f.acc_splits = acc.data_ptr(), splits
    N.factor_flush([f], hip_device)
    want = F0.astype(np.float64)
    for x in xs:
        xo = np.concatenate([x, np.ones((x.shape[0], 1), np.float32)], 1).astype(np.float64)
        want += xo.T @ xo
    np.testing.assert_array_equal(F.cpu().numpy(), want)


def test_split_accumulator_ranges_raw_abi(hip_device):
    """Two jobs of ONE factor in ONE kfac_factor_update call, each accumulating into its
    own split-K slab range (acc = base + s0 slabs, acc_stride = the factor's total), then
    one kfac_factor_flush over all slabs (include/kfac_hip.h, acc_stride): F0 + both
    batches, exact on small integers, for the fp32-MFMA (129) and bf16x3 (785) kernels.
    An acc_stride below acc_splits is rejected before any launch."""
    from bnn_kfac_amd import _native as N
    rng = np.random.default_rng(11)
    slab = 64 * 64 * 4
    for cols in (128, 784):
        n = cols + 1
        F0 = rng.integers(-4, 5, size=(n, n)).astype(np.float32)
        F0 = F0 + F0.T
        F = _t(F0, hip_device)
        xs = [rng.integers(-3, 4, size=(B, cols)).astype(np.float32) for B in (4096, 608)]
        xd = [_t(x, hip_device) for x in xs]
        jobs = [N.factor_job(N.rowmajor_operand(x, True), F, 1.0, 1.0) for x in xd]
        plan = N.factor_accum_plan(jobs)
        total = sum(sp for sp, _ in plan)
        acc = torch.empty(sum(nb for _, nb in plan), dtype=torch.uint8, device=hip_device)
        s0 = 0
        for j, (sp, _) in zip(jobs, plan):
            j.acc, j.acc_splits, j.acc_beta, j.acc_stride = acc.data_ptr() + s0 * slab, sp, 0.0, total
            s0 += sp
        bad = N.FactorJob.from_buffer_copy(jobs[0])
        bad.acc_stride = max(1, bad.acc_splits - 1) if bad.acc_splits > 1 else -1
        with pytest.raises(N.NativeError):
            N.factor_update([bad], hip_device)
        N.factor_update(jobs, hip_device)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(F.cpu().numpy(), F0)
        f = N.factor_job(N.rowmajor_operand(xd[0], True), F, 1.0, 1.0)
        f.acc, f.acc_splits, f.acc_stride = acc.data_ptr(), total, total
        N.factor_flush([f], hip_device)
        want = F0.astype(np.float64)
        for x in xs:
            xo = np.concatenate([x, np.ones((x.shape[0], 1), np.float32)], 1).astype(np.float64)
            want += xo.T @ xo
        np.testing.assert_array_equal(F.cpu().numpy(), want)


@pytest.mark.parametrize("cols,rows,offset,ones", [(784, 4096, 0, True), (128, 1000, 0, False),
                                                    (129, 333, 0, True), (10, 4096, 0, False),
                                                    (96, 777, 1, True), (31, 65, 0, True)])
@pytest.mark.parametrize("deferred", [False, True])
def test_multibatch_job_raw_abi(hip_device, cols, rows, offset, ones, deferred):
    """One multi-batch job (nseg batches, each its own allocation, read in place
    through the bases passed as kernel arguments) equals the sum over the batches, exactly on
    small integers: LDS-DMA (aligned), register-staged (odd width / unaligned base)
    and narrow (n <= 32) paths, ragged last stages, with and without accumulators."""
    from bnn_kfac_amd import _native as N
    rng = np.random.default_rng(cols + rows)
    nseg = 5
    xs = [rng.integers(-3, 4, size=(rows, cols)).astype(np.float32) for _ in range(nseg)]
    # separate allocations; `offset` floats into each so every base has the same misalignment
    bufs = [torch.empty(rows * cols + 8, device=hip_device) for _ in range(nseg)]
    views = []
    for b, x in zip(bufs, xs):
        v = b[offset:offset + rows * cols].view(rows, cols)
        v.copy_(_t(x, hip_device))
        views.append(v)
    n = cols + ones
    F = torch.full((n, n), np.nan, device=hip_device)
    table = N.segment_table([v.data_ptr() for v in views])
    job = N.factor_job(N.rowmajor_operand(views[0], ones), F, 1.0, 0.0)
    job.seg_ptrs, job.nseg = N.table_ptr(table), nseg
    if deferred:
        (splits, nbytes), = N.factor_accum_plan([job])
        acc = torch.empty(nbytes, dtype=torch.uint8, device=hip_device)
        job.acc, job.acc_splits, job.acc_beta = acc.data_ptr(), splits, 0.0
        N.factor_update([job], hip_device)
        f = N.factor_job(N.rowmajor_operand(views[0], ones), F, 1.0, 0.0)
        f.acc, f.acc_splits = acc.data_ptr(), splits
        N.factor_flush([f], hip_device)
    else:
        N.factor_update([job], hip_device)
    want = np.zeros((n, n))
    for x in xs:
        xo = np.concatenate([x, np.ones((rows, 1), np.float32)], 1) if ones else x
        want += xo.T.astype(np.float64) @ xo
    np.testing.assert_array_equal(F.cpu().numpy(), want)


@pytest.mark.parametrize("deferred", [False, True])
def test_x3_thin_row_pairs_exact(hip_device, deferred):
    """kfac_factor_tiles_x3's work units (one launch: the group's largest factor, 785,
    selects it; every operand 16-byte rows): factors whose last tile row is thin (785:
    17 rows, 129: 1, 93: 29, 65: 1) run their diagonal tiles paired with the edge tiles
    below them, 97 (33 rows), 128 and 33 (one tile) do not; multi-batch operands with a
    ragged last stage; exact on small integers against the fp64 sum."""
    from bnn_kfac_amd import _native as N
    rng = np.random.default_rng(7)
    nseg, rows = 3, 1000
    cases = [(784, True), (128, True), (92, True), (64, True), (96, True), (32, True), (128, False)]
    jobs, want, keep, outs, accs = [], [], [], [], []
    for cols, ones in cases:
        xs = [rng.integers(-3, 4, size=(rows, cols)).astype(np.float32) for _ in range(nseg)]
        views = [_t(x, hip_device) for x in xs]
        keep.append(views)
        n = cols + ones
        F = torch.full((n, n), np.nan, device=hip_device)
        outs.append(F)
        table = N.segment_table([v.data_ptr() for v in views])
        keep.append(table)
        job = N.factor_job(N.rowmajor_operand(views[0], ones), F, 1.0, 0.0)
        job.seg_ptrs, job.nseg = N.table_ptr(table), nseg
        jobs.append(job)
        w = np.zeros((n, n))
        for x in xs:
            xo = np.concatenate([x, np.ones((rows, 1), np.float32)], 1) if ones else x
            w += xo.T.astype(np.float64) @ xo
        want.append(w)
    N.profile_reset()
    N.profile_enable(True)
    if deferred:
        plan = N.factor_accum_plan(jobs)
        flush = []
        for job, (splits, nbytes) in zip(jobs, plan):
            acc = torch.empty(nbytes, dtype=torch.uint8, device=hip_device)
            accs.append(acc)
            job.acc, job.acc_splits, job.acc_beta = acc.data_ptr(), splits, 0.0
            f = N.FactorJob.from_buffer_copy(job)
            f.seg_ptrs, f.nseg = None, 0
            flush.append(f)
        N.factor_update(jobs, hip_device)
        N.factor_flush(flush, hip_device)
    else:
        N.factor_update(jobs, hip_device)
    torch.cuda.synchronize()
    N.profile_enable(False)
    assert N.profile_read(N.PROF_FACTOR_X3)[1] == 1  # one kfac_factor_tiles_x3 launch
    for F, w in zip(outs, want):
        np.testing.assert_array_equal(F.cpu().numpy(), w)


@pytest.mark.parametrize("deferred", [False, True])
def test_x3_pair_extra_splits_exact(hip_device, deferred):
    """Thin-row pair units take S/11 extra, shorter K-splits of S slabs per tile (the
    full tiles' last K-split writes zero partials into those slabs): a 785 factor (pairs)
    beside a 128 one (no pairs) over 8 batches of 4096 rows, planned at S >= 11, exact on
    small integers against the fp64 sum, immediate and deferred."""
    from bnn_kfac_amd import _native as N
    rng = np.random.default_rng(13)
    nseg, rows = 8, 4096
    jobs, want, keep, outs, accs = [], [], [], [], []
    for cols, ones in ((784, True), (128, False)):
        xs = [rng.integers(-2, 3, size=(rows, cols)).astype(np.float32) for _ in range(nseg)]
        views = [_t(x, hip_device) for x in xs]
        keep.append(views)
        n = cols + ones
        F = torch.full((n, n), np.nan, device=hip_device)
        outs.append(F)
        table = N.segment_table([v.data_ptr() for v in views])
        keep.append(table)
        job = N.factor_job(N.rowmajor_operand(views[0], ones), F, 1.0, 0.0)
        job.seg_ptrs, job.nseg = N.table_ptr(table), nseg
        jobs.append(job)
        w = np.zeros((n, n))
        for x in xs:
            xo = np.concatenate([x, np.ones((rows, 1), np.float32)], 1) if ones else x
            w += xo.T.astype(np.float64) @ xo
        want.append(w)
    plan = N.factor_accum_plan(jobs)
    assert plan[0][0] >= 11, plan  # the 785 factor's pair units get extra K-splits
    if deferred:
        flush = []
        for job, (splits, nbytes) in zip(jobs, plan):
            acc = torch.empty(nbytes, dtype=torch.uint8, device=hip_device)
            accs.append(acc)
            job.acc, job.acc_splits, job.acc_beta = acc.data_ptr(), splits, 0.0
            f = N.FactorJob.from_buffer_copy(job)
            f.seg_ptrs, f.nseg = None, 0
            flush.append(f)
        N.factor_update(jobs, hip_device)
        N.factor_flush(flush, hip_device)
    else:
        N.factor_update(jobs, hip_device)
    torch.cuda.synchronize()
    for F, w in zip(outs, want):
        np.testing.assert_array_equal(F.cpu().numpy(), w)


def test_queued_pass_matches_per_batch_launches(hip_device):
    """KFAC's default queued pass (multi-batch jobs, one short last batch, separate
    record allocations) equals launching every update on its own."""
    from bnn_kfac_amd.curvatures import KFAC
    torch.manual_seed(0)
    net = nn.Sequential(nn.Linear(784, 128), nn.ReLU(), nn.Linear(128, 10)).to(hip_device)
    g = torch.Generator(device=hip_device).manual_seed(2)
    recs = [(torch.rand(B, 784, device=hip_device, generator=g), torch.rand(B, 128, device=hip_device, generator=g),
             torch.randn(B, 128, device=hip_device, generator=g), torch.randn(B, 10, device=hip_device, generator=g))
            for B in (4096,) * 6 + (1700,)]
    from bnn_kfac_amd import _native as N
    outs = []
    orig = N.factor_update
    # (defer_batches, launch_first, merge_launches): per update; doubling launches; the
    # whole pass queued as one flush: 6 full batches and the short one as their ragged
    # last batch, one launch (merge_launches has one group left to merge)
    for defer_batches, first, merge in ((1, 1, False), (64, 1, False), (4, 1, False), (64, 16, False),
                                        (64, 16, True)):
        kfac = KFAC(net)
        kfac.defer_batches = defer_batches
        kfac.launch_first = first
        kfac.merge_launches = merge
        calls = []

        def counting(jobs, device):
            calls.append(len(jobs))
            return orig(jobs, device)
        N.factor_update = counting
        try:
            for a1, a2, g1, g2 in recs:
                kfac.record[net[0]] = [a1, g1]
                kfac.record[net[2]] = [a2, g2]
                kfac.update(a1.shape[0])
            outs.append([t.cpu().numpy() for pair in kfac.state.values() for t in pair])
        finally:
            N.factor_update = orig
        if first == 16:
            # the short batch rides as the ragged last batch (x.last_rows) of the full
            # batches' jobs: one group, one launch
            assert calls == [4], calls
    for other in outs[1:]:
        for got, want in zip(other, outs[0]):
            np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6 * np.abs(want).max())
    ref = O.OracleKFAC(np.float64)
    for a1, a2, g1, g2 in recs:
        ref.update_linear("l0", a1.cpu().numpy(), g1.cpu().numpy(), True)
        ref.update_linear("l1", a2.cpu().numpy(), g2.cpu().numpy(), True)
    for got, want in zip(outs[1], [t for k in ("l0", "l1") for t in ref.state[k]]):
        np.testing.assert_allclose(got, want, **FT)


@pytest.mark.parametrize("model", ["mlp", "lenet"])
def test_deferred_reduce_matches_immediate(hip_device, model):
    """KFAC.update with the deferred reduction (default) equals the per-update
    reduce, for row-major and conv factors, across a mid-pass `state` read."""
    from bnn_kfac_amd.curvatures import KFAC
    torch.manual_seed(0)
    if model == "mlp":
        net = nn.Sequential(nn.Linear(784, 128), nn.ReLU(), nn.Linear(128, 10)).to(hip_device)
        shape = (784,)
    else:
        net = nn.Sequential(nn.Conv2d(1, 6, 5), nn.ReLU(), nn.MaxPool2d(2), nn.Conv2d(6, 16, 5),
                            nn.ReLU(), nn.MaxPool2d(2), nn.Flatten(), nn.Linear(256, 10)).to(hip_device)
        shape = (1, 28, 28)
    g = torch.Generator(device=hip_device).manual_seed(1)
    xs = [torch.rand(B, *shape, device=hip_device, generator=g) for B in (1024, 1024, 300, 1024)]
    outs = []
    for defer, read_at in ((False, -1), (True, -1), (True, 1)):
        kfac = KFAC(net)
        kfac.defer_reduce = defer
        for i, x in enumerate(xs):
            out = net(x)
            net.zero_grad()
            nn.functional.cross_entropy(out, out.argmax(1)).backward()
            kfac.update(x.shape[0])
            if i == read_at:
                _ = kfac.state
        outs.append([t.cpu().numpy() for pair in kfac.state.values() for t in pair])
        for h in kfac.hooks:
            h.remove()
    for other in outs[1:]:
        for got, want in zip(other, outs[0]):
            np.testing.assert_allclose(got, want, rtol=1e-5, atol=1e-6 * np.abs(want).max())


@pytest.mark.parametrize("spec", [
    # (B, Cin, H, W, Cout, k, stride, pad, bias): LeNet-5's conv1 / conv2 (n <= 8 channel
    # kernel, staged im2col), a 32-wide channel factor with a narrow im2col one, and an
    # image too large to stage (multi-batch job split into per-batch launches)
    (64, 1, 28, 28, 6, (5, 5), (1, 1), (2, 2), True),
    (32, 6, 14, 14, 16, (5, 5), (1, 1), (0, 0), True),
    (4, 1, 10, 10, 20, (3, 3), (1, 1), (1, 1), True),
    (2, 3, 40, 40, 5, (3, 3), (1, 1), (1, 1), True),
])
@pytest.mark.parametrize("deferred", [False, True])
def test_conv_multibatch_queue_vs_oracle(hip_device, spec, deferred):
    """Queued Conv2d updates become ONE multi-batch job per factor (the images walk
    the batches' bases): 7 batches of separate allocations plus a short last one,
    queued through KFAC.update, against the fp64 oracle's sum of per-batch means."""
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import KFAC
    B, Cin, H, W, Cout, k, s, p, bias = spec
    rng = np.random.default_rng(sum(spec[:5]) + 7)
    conv = nn.Conv2d(Cin, Cout, k, stride=s, padding=p, bias=bias).to(hip_device)
    Ho, Wo = (H + 2 * p[0] - k[0]) // s[0] + 1, (W + 2 * p[1] - k[1]) // s[1] + 1
    sizes = [B] * 7 + [max(1, B // 3)]
    xs = [rng.random((b, Cin, H, W), dtype=np.float32) for b in sizes]
    gs = [rng.standard_normal((b, Cout, Ho, Wo), dtype=np.float32) for b in sizes]
    kfac = KFAC(conv)
    kfac.defer_reduce = deferred
    kfac.launch_first = 8
    calls = []
    orig = N.factor_update

    def counting(jobs, device):
        calls.append([max(1, j.nseg) for j in jobs])
        return orig(jobs, device)
    N.factor_update = counting
    try:
        for x, g in zip(xs, gs):
            kfac.record[conv] = [_t(x, hip_device), _t(g, hip_device)]
            kfac.update(batch_size=x.shape[0])
        A, G = kfac.state[conv]
    finally:
        N.factor_update = orig
    if deferred:
        # the 7 equal batches: one job per factor (the short batch's jobs follow in the
        # same launch when merge_launches holds, else in a launch of their own)
        assert calls[0][:2] == [7, 7], calls
    wA = sum(O.conv_factor_A(x, k, p, s, bias, np.float64) for x in xs)
    wG = sum(O.grad_factor(g, np.float64) for g in gs)
    np.testing.assert_allclose(A.cpu().numpy(), wA, **FT)
    np.testing.assert_allclose(G.cpu().numpy(), wG, **FT)
