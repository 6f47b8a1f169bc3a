"""A pass's short last batch as the ragged last segment of the multi-batch jobs
(kfac_operand.last_rows): every batch still enters as its own per-batch mean
(models/curvatures.py:349,356: `/ forward.shape[1]`, summed over updates at
:359-363), the last one weighed rows / last_rows against the full ones inside the
launch (a task crossing into it rescales its sums at the boundary).

Through KFAC.update with the whole pass queued (launch_first 16): the MNIST MLP's
bf16x3 path (kfac_factor_tiles_x3 + its narrow n <= 32 tasks, thin-row pairs, the
ones column), last batches that are / are not a multiple of the 32-row stage, and a
small MLP whose fp32-kernel launch group the library splits into two launches.
Every A / G against the fp64 oracle's sum of per-batch means at rtol 1e-5.
"""
import numpy as np
import pytest
import torch

from oracle import kfac_oracle as O

pytestmark = pytest.mark.gpu


def _pass(net, batches, launch_first=16, defer=True):
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import KFAC
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    kfac = KFAC(net)
    kfac.launch_first = launch_first
    kfac.defer_reduce = defer
    seen = []
    orig = N.factor_update

    def spy(jobs, device):
        seen.append([(j.nseg, j.x.last_rows) for j in jobs])
        return orig(jobs, device)
    N.factor_update = spy
    try:
        for recs in batches:
            for layer, (a, g) in zip(layers, recs):
                kfac.record[layer] = [a, g]
            kfac.update(recs[0][0].shape[0])
        state = [[t.double().cpu().numpy() for t in kfac.state[m]] for m in layers]
    finally:
        N.factor_update = orig
    return state, seen


def _oracle(batches):
    out = []
    for li in range(len(batches[0])):
        A = sum(O.linear_factor_A(b[li][0].cpu().numpy(), True, np.float64) for b in batches)
        G = sum(O.grad_factor(b[li][1].cpu().numpy(), np.float64) for b in batches)
        out.append((A, G))
    return out


def _batches(dims, sizes, dev, seed):
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    return [[(torch.rand(B, d_in, device=dev, generator=g), torch.randn(B, d_out, device=dev, generator=g))
             for d_in, d_out in dims] for B in sizes]


@pytest.mark.parametrize("last", [2656, 608, 33, 1])
def test_ragged_last_batch_mlp_x3(hip_device, last):
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(784, 128), torch.nn.ReLU(), torch.nn.Linear(128, 10)).to(hip_device)
    batches = _batches([(784, 128), (128, 10)], [4096] * 5 + [last], hip_device, seed=last)
    state, seen = _pass(net, batches)
    assert seen == [[(6, last)] * 4], seen  # one launch, the short batch ragged
    for li, ((A, G), (wA, wG)) in enumerate(zip(state, _oracle(batches))):
        for name, got, ref in (("A", A, wA), ("G", G, wG)):
            np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max(),
                                       err_msg=f"layer {li} {name} last={last}")


@pytest.mark.parametrize("defer", [True, False])
def test_ragged_last_batch_split_for_fp32_kernel(hip_device, defer):
    """n < 512: the fp32-MFMA launch group takes the ragged job as two launches."""
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(40, 24), torch.nn.ReLU(), torch.nn.Linear(24, 6)).to(hip_device)
    batches = _batches([(40, 24), (24, 6)], [512] * 3 + [77], hip_device, seed=3)
    state, seen = _pass(net, batches, defer=defer)
    if defer:
        assert seen == [[(4, 77)] * 4], seen
    for li, ((A, G), (wA, wG)) in enumerate(zip(state, _oracle(batches))):
        for name, got, ref in (("A", A, wA), ("G", G, wG)):
            np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max(),
                                       err_msg=f"layer {li} {name}")


def test_ragged_serial_launch_doubling(hip_device):
    """The serial loop's launch sizes (1, 2, 4, 8: the last launch 7 full batches +
    the short one) over 15 batches, against the fp64 oracle."""
    torch.manual_seed(0)
    net = torch.nn.Sequential(torch.nn.Linear(784, 128), torch.nn.ReLU(), torch.nn.Linear(128, 10)).to(hip_device)
    batches = _batches([(784, 128), (128, 10)], [4096] * 14 + [2656], hip_device, seed=9)
    state, seen = _pass(net, batches, launch_first=1)
    assert seen[-1] == [(8, 2656)] * 4, seen
    for li, ((A, G), (wA, wG)) in enumerate(zip(state, _oracle(batches))):
        for name, got, ref in (("A", A, wA), ("G", G, wG)):
            np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max(),
                                       err_msg=f"layer {li} {name}")
