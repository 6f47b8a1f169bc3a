"""GPU: the reference-side binding of INTEGRATION.md §2, exercised exactly as a
maintainer would add it next to models/curvatures.py.

The stub below is INTEGRATION.md's ctypes code (plus its conv siblings from
include/kfac_hip.h): a fresh ctypes.CDLL handle on libkfac_hip.so, plain pointers,
sizes and the torch stream -- none of bnn_kfac_amd's own Python.  It replaces

* the Linear branch of KFAC.update (curvatures.py:345-349, 355-356) -> kfac_syrk_linear,
* the Conv2d F.unfold branch (:341-343) -> kfac_syrk_conv,
* the Conv2d grad permute branch (:352-353) -> kfac_syrk_convgrad,
* the "+=" of :359-363 -> beta = 1,
* KFAC.invert's inverse().cholesky() (:381-396) -> kfac_damped_inv_chol,

and is driven by the reference's own outputs: G1 (MLP factors and L factors), G1
small (three damping forms), G4 (conv factors, two updates) and G2 (the singular
factor: info > 0 where the reference falls into its numpy path and raises).

Tolerances: factors rtol 1e-5 (fp32 sums, as tests/test_gpu_factors.py); L factors
rtol 1e-4 against the fp64 oracle on the same factor (the north-star figure), and
the reference's own fp32 band against its fixtures (as tests/test_gpu_invert.py).
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from conftest import ROOT, golden
from oracle import kfac_oracle as O

pytestmark = pytest.mark.gpu

# ---------------------------------------------------------------- the stub
_lib = ctypes.CDLL(os.path.join(ROOT, "bnn_kfac_amd", "libkfac_hip.so"))
_vp, _i64, _f32, _f64, _i = ctypes.c_void_p, ctypes.c_int64, ctypes.c_float, ctypes.c_double, ctypes.c_int
_lib.kfac_syrk_linear.argtypes = [_vp, _i64, _i64, _i64, _i, _f32, _f32, _vp, _i64, _vp, ctypes.c_size_t, _vp]
_lib.kfac_syrk_conv.argtypes = [_vp, _i64, _i, _i, _i, _i, _i, _i, _i, _i, _i, _i, _f32, _f32, _vp, _i64,
                                _vp, ctypes.c_size_t, _vp]
_lib.kfac_syrk_convgrad.argtypes = [_vp, _i64, _i, _i64, _f32, _f32, _vp, _i64, _vp, ctypes.c_size_t, _vp]
_lib.kfac_damped_inv_chol.argtypes = [_vp, _i, _i64, _f64, _f64, _vp, _i64, _vp, ctypes.c_size_t, _vp, _vp]
_lib.kfac_strerror.restype = ctypes.c_char_p
WS = 64 << 20  # caller-owned workspace; kfac_*_workspace_bytes() give exact sizes


def _stream(t):
    return torch.cuda.current_stream(t.device).cuda_stream


def _ok(rc):
    if rc != 0:
        raise RuntimeError(_lib.kfac_strerror(rc).decode())


def syrk_linear(x, has_ones, alpha, beta, F, ws):
    """F = beta*F + alpha*[x^T;1^T][x^T;1^T]^T   (curvatures.py:345-349 / 355-356, 359-363)"""
    _ok(_lib.kfac_syrk_linear(x.data_ptr(), x.shape[0], x.shape[1], x.stride(0), int(has_ones),
                              alpha, beta, F.data_ptr(), F.stride(0), ws.data_ptr(), ws.numel(),
                              _vp(_stream(x))))


def syrk_conv(x, layer, alpha, beta, F, ws):
    """F = beta*F + alpha*U U^T, U = [unfold(x) rows; 1^T]   (curvatures.py:341-343, 347-349)"""
    B, C, H, W = x.shape
    (kh, kw), (sh, sw), (ph, pw) = layer.kernel_size, layer.stride, layer.padding
    _ok(_lib.kfac_syrk_conv(x.data_ptr(), B, C, H, W, kh, kw, sh, sw, ph, pw, int(layer.bias is not None),
                            alpha, beta, F.data_ptr(), F.stride(0), ws.data_ptr(), ws.numel(),
                            _vp(_stream(x))))


def syrk_convgrad(g, alpha, beta, F, ws):
    """F = beta*F + alpha*P P^T, P = g.permute(1,0,2,3).view(C, -1)   (curvatures.py:352-356)"""
    B, C, Ho, Wo = g.shape
    _ok(_lib.kfac_syrk_convgrad(g.data_ptr(), B, C, Ho * Wo, alpha, beta, F.data_ptr(), F.stride(0),
                                ws.data_ptr(), ws.numel(), _vp(_stream(g))))


def damped_inv_chol(F, s, n, L, ws, info):
    """L = cholesky(inverse((sqrt(s)F + sqrt(n)I + transpose)/2))   (curvatures.py:381-391)"""
    _ok(_lib.kfac_damped_inv_chol(F.data_ptr(), F.shape[0], F.stride(0), s ** 0.5, n ** 0.5,
                                  L.data_ptr(), L.stride(0), ws.data_ptr(), ws.numel(),
                                  info.data_ptr(), _vp(_stream(F))))
    if int(info.item()) != 0:                    # > 0: leading minor not positive definite
        raise RuntimeError("cholesky: not positive definite")   # -> the reference's numpy fallback
# ---------------------------------------------------------------- end of the stub


FT = dict(rtol=1e-5, atol=1e-6)


def _t(x, dev):
    return torch.from_numpy(np.ascontiguousarray(x)).to(dev)


@pytest.fixture
def ws(hip_device):
    return torch.empty(WS, dtype=torch.uint8, device=hip_device)


def _mlp_batches(seed=123, sizes=(256, 256, 256, 96)):  # tests/golden/make_goldens.py mlp_batches
    rng = np.random.default_rng(seed)
    for B in sizes:
        yield (B, rng.random((B, 784), dtype=np.float32), rng.standard_normal((B, 128), dtype=np.float32),
               rng.random((B, 128), dtype=np.float32), rng.standard_normal((B, 10), dtype=np.float32))


def test_stub_mlp_update_and_invert(hip_device, ws):
    """G1: the reference's MLP factors over four batches (the last one short) and its L
    factors at the classification scripts' damping, through the stub alone."""
    g = golden("g1_mlp.npz")
    F = [torch.empty(n, n, device=hip_device) for n in (785, 128, 129, 10)]
    for b, (B, a1, g1, a2, g2) in enumerate(_mlp_batches()):
        beta = 0.0 if b == 0 else 1.0
        for x, ones, Fi in ((a1, True, F[0]), (g1, False, F[1]), (a2, True, F[2]), (g2, False, F[3])):
            syrk_linear(_t(x, hip_device), ones, 1.0 / B, beta, Fi, ws)
    A1, G1, A2, G2 = [f.cpu().numpy() for f in F]
    np.testing.assert_allclose(np.diag(A1), g["A1_diag"], **FT)
    np.testing.assert_allclose(A1[:8], g["A1_head"], **FT)
    np.testing.assert_allclose(A1[-8:], g["A1_tail"], **FT)
    np.testing.assert_allclose(G1, g["G1"], **FT)
    np.testing.assert_allclose(A2, g["A2"], **FT)
    np.testing.assert_allclose(G2, g["G2"], **FT)
    assert all(np.array_equal(f, f.T) for f in (A1, G1, A2, G2))
    info = torch.zeros(1, dtype=torch.int32, device=hip_device)
    Ls = []
    for Fi in F:
        L = torch.full_like(Fi, float("nan"))
        damped_inv_chol(Fi, 200.0, 0.2 ** 2, L, ws, info)  # invert(add=0.04, multiply=200)
        Ls.append(L.cpu().numpy())
    for L, Fh in zip(Ls, (A1, G1, A2, G2)):
        np.testing.assert_allclose(L, O.invert_factor(Fh, 0.04, 200), rtol=1e-4, atol=1e-7)
        assert np.all(np.triu(L, 1) == 0)
    np.testing.assert_allclose(Ls[1], g["LG1"], rtol=5e-4, atol=1e-5)
    np.testing.assert_allclose(Ls[2], g["LA2"], rtol=5e-4, atol=1e-5)
    np.testing.assert_allclose(Ls[3], g["LG2"], rtol=5e-4, atol=1e-5)
    np.testing.assert_allclose(np.diag(Ls[0]), g["LA1_diag"], rtol=1e-2, atol=1e-5)


def test_stub_small_linear_damping_forms(hip_device, ws):
    """G1 small: a layer without bias, the short last batch, and the reference's three
    damping forms (the script's, the tutorial's and a per-layer list)."""
    g = golden("g1_small_linear.npz")
    F = {k: torch.empty(n, n, device=hip_device) for k, n in (("A0", 21), ("G0", 12), ("A1", 12), ("G1", 5))}
    for bi in range(3):
        B = len(g[f"b{bi}_a1"])
        beta = 0.0 if bi == 0 else 1.0
        syrk_linear(_t(g[f"b{bi}_a1"], hip_device), True, 1.0 / B, beta, F["A0"], ws)
        syrk_linear(_t(g[f"b{bi}_g1"], hip_device), False, 1.0 / B, beta, F["G0"], ws)
        syrk_linear(_t(g[f"b{bi}_a2"], hip_device), False, 1.0 / B, beta, F["A1"], ws)  # bias=False
        syrk_linear(_t(g[f"b{bi}_g2"], hip_device), False, 1.0 / B, beta, F["G1"], ws)
    for k, Fk in F.items():
        np.testing.assert_allclose(Fk.cpu().numpy(), g[k], **FT)
    info = torch.zeros(1, dtype=torch.int32, device=hip_device)
    for tag, (add, mult) in {"s": ((0.04, 0.04), (200, 200)), "t": ((1, 1), (200, 200)),
                             "l": ((0.1, 0.3), (10.0, 20.0))}.items():
        for li in range(2):
            for kind in ("A", "G"):
                Fk = F[f"{kind}{li}"]
                L = torch.empty_like(Fk)
                damped_inv_chol(Fk, float(mult[li]), float(add[li]), L, ws, info)
                got = L.cpu().numpy()
                want = O.invert_factor(Fk.cpu().numpy(), add[li], mult[li])
                np.testing.assert_allclose(got, want, rtol=1e-4, atol=1e-8)
                np.testing.assert_allclose(got, g[f"inv{tag}_L{kind}{li}"], rtol=2e-4, atol=2e-5)


def test_stub_conv_factors(hip_device, ws):
    """G4: four Conv2d layers (BaseNet_750's two, a padded LeNet-5-style one and an
    asymmetric-kernel, strided one without bias), two updates (the "+=")."""
    g = golden("g4_conv.npz")
    for li in range(4):
        kh, kw, sh, sw, ph, pw, bias, cout = [int(v) for v in g[f"meta{li}"]]
        x = _t(g[f"x{li}"], hip_device)
        gr = _t(g[f"g{li}"], hip_device)
        layer = torch.nn.Conv2d(x.shape[1], cout, (kh, kw), stride=(sh, sw), padding=(ph, pw), bias=bool(bias))
        nA = x.shape[1] * kh * kw + int(bool(bias))
        A = torch.empty(nA, nA, device=hip_device)
        G = torch.empty(cout, cout, device=hip_device)
        rows = gr.shape[0] * gr.shape[2] * gr.shape[3]  # forward.shape[1] = B * L
        for u in range(2):
            syrk_conv(x, layer, 1.0 / rows, float(u), A, ws)
            syrk_convgrad(gr, 1.0 / rows, float(u), G, ws)
        np.testing.assert_allclose(A.cpu().numpy(), g[f"A{li}"], **FT)
        np.testing.assert_allclose(G.cpu().numpy(), g[f"G{li}"], **FT)


def test_stub_singular_factor(hip_device, ws):
    """G2: invert(0, 1) of a rank-2 7x7 factor.  The reference's torch cholesky fails
    and its numpy fallback raises LinAlgError; through the stub, info > 0 (the first
    non-positive pivot + 1) and the stub raises."""
    g = golden("g2_singular.npz")
    assert str(g["outcome"]) == "LinAlgError"
    A = torch.empty(7, 7, device=hip_device)
    syrk_linear(_t(g["a"], hip_device), True, 0.5, 0.0, A, ws)
    np.testing.assert_allclose(A.cpu().numpy(), g["A"], **FT)
    info = torch.zeros(1, dtype=torch.int32, device=hip_device)
    L = torch.empty_like(A)
    with pytest.raises(RuntimeError, match="not positive definite"):
        damped_inv_chol(A, 1.0, 0.0, L, ws, info)
    assert 1 <= int(info.item()) <= 7
    damped_inv_chol(A, 1.0, 1.0, L, ws, info)  # damped: positive definite
    np.testing.assert_allclose(L.cpu().numpy(), O.invert_factor(A.cpu().numpy(), 1.0, 1.0),
                               rtol=1e-4, atol=1e-8)


def test_stub_rejects_bad_arguments(hip_device, ws):
    """Status codes come back synchronously: a too-small workspace and a negative size."""
    x = torch.rand(64, 785, device=hip_device)
    F = torch.empty(786, 786, device=hip_device)
    with pytest.raises(RuntimeError, match="workspace"):
        _ok(_lib.kfac_syrk_linear(x.data_ptr(), 64, 785, 785, 1, 1.0, 0.0, F.data_ptr(), 786,
                                  ws.data_ptr(), 16, _vp(_stream(x))))
    with pytest.raises(RuntimeError, match="invalid"):
        _ok(_lib.kfac_syrk_linear(x.data_ptr(), -1, 785, 785, 1, 1.0, 0.0, F.data_ptr(), 786,
                                  ws.data_ptr(), ws.numel(), _vp(_stream(x))))
