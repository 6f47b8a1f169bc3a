"""GPU parity at BASELINE C3's stated config: bench.py's exact LeNet-5 (conv1 1->6 k5
p2, conv2 6->16 k5, fc 400-120-84-10) at batch 1024 over one MNIST-sized pass of
60,000 images (58 full batches + a 608-row last batch), through the default
KFAC.update path -- queued multi-batch launches, the conv planner's images-per-task
choice at B = 1024, the n <= 8 channel kernel, deferred reduction -- then
invert(0.04, 200) (classification_ll_block.py:72-73,106).

Every A / G against the fp64 oracle (models/curvatures.py:341-363: O.conv_factor_A,
O.linear_factor_A, O.grad_factor summed over the batches) at rtol 1e-5, and every
L against O.invert_factor (curvatures.py:381-398) on the device's own factor within
1e-4 of max|L|.
"""
import numpy as np
import pytest
import torch

import bench
from oracle import kfac_oracle as O

pytestmark = pytest.mark.gpu

IMAGES, BATCH = 60000, 1024


def _oracle_pass(specs, recs_cpu):
    """fp64 state of one pass (sum of per-batch means), batch by batch."""
    state = []
    for l, (x, g) in zip(specs, recs_cpu):
        A = G = 0.0
        for i in range(0, IMAGES, BATCH):
            xb, gb = x[i:i + BATCH], g[i:i + BATCH]
            if l.kind == "linear":
                A = A + O.linear_factor_A(xb, True, np.float64)
            else:
                A = A + O.conv_factor_A(xb, (l.k, l.k), (l.pad, l.pad), (l.stride, l.stride), True,
                                        np.float64)
            G = G + O.grad_factor(gb, np.float64)
        state.append((A, G))
    return state


def test_lenet5_c3_pass_and_invert_vs_fp64_oracle(hip_device):
    from bnn_kfac_amd.curvatures import KFAC
    assert IMAGES % BATCH == 608
    specs = bench.CONFIGS["lenet"]
    net = bench.build_model("lenet", hip_device)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    assert [tuple(m.weight.shape) for m in layers] == [(6, 1, 5, 5), (16, 6, 5, 5), (120, 400),
                                                        (84, 120), (10, 84)]
    recs = bench.synthetic_records(specs, IMAGES, hip_device, seed=77)
    kfac = KFAC(net)
    launches = []
    from bnn_kfac_amd import _native as N
    orig = N.factor_update

    def counting(jobs, device):
        launches.append(len(jobs))
        return orig(jobs, device)
    N.factor_update = counting
    try:
        kfac.reset()
        for i in range(0, IMAGES, BATCH):  # bench.py one_pass
            for layer, (a, g) in zip(layers, recs):
                kfac.record[layer] = [a[i:i + BATCH], g[i:i + BATCH]]
            kfac.update(batch_size=min(BATCH, IMAGES - i))
        kfac.invert(0.2 ** 2, 200)
    finally:
        N.factor_update = orig
    # queued: far fewer factor_update calls than the 59 updates, more than one
    assert 1 < len(launches) < 59, launches
    state = [[t.cpu().numpy() for t in kfac.state[m]] for m in layers]
    inv = [[t.cpu().numpy() for t in kfac.inv_state[m]] for m in layers]
    recs_cpu = [(a.cpu().numpy(), g.cpu().numpy()) for a, g in recs]
    del recs
    want = _oracle_pass(specs, recs_cpu)
    for li, ((A, G), (wA, wG)) in enumerate(zip(state, want)):
        for name, got, ref in (("A", A, wA), ("G", G, wG)):
            np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max(),
                                       err_msg=f"layer {li} {name}")
    for li, ((A, G), (LA, LG)) in enumerate(zip(state, inv)):
        for name, F, L in (("L_A", A, LA), ("L_G", G, LG)):
            ref = O.invert_factor(F.astype(np.float64), 0.04, 200)
            np.testing.assert_allclose(L, ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max(),
                                       err_msg=f"layer {li} {name}")
            assert np.all(np.triu(L, 1) == 0)


@pytest.mark.parametrize("config", ["lenet", "mlp"])
def test_repeated_passes_fast_path_bit_identical(hip_device, config):
    """The bench's loop (reset, a pass of updates with a short last batch, invert) four
    times over the same records: from the third pass on no update takes the slow path
    (cached per-buffer templates start each cycle, the short batch has its own), the
    double-buffered state alternates, and every pass's factors and L factors are
    bit-identical to the first pass's (deterministic kernels, same inputs)."""
    from bnn_kfac_amd.curvatures import KFAC
    images, batch = (8 * 1024 + 300, 1024) if config == "lenet" else (6 * 4096 + 1000, 4096)
    specs = bench.CONFIGS[config]
    net = bench.build_model(config, hip_device)
    layers = [m for m in net.modules() if isinstance(m, (torch.nn.Linear, torch.nn.Conv2d))]
    recs = bench.synthetic_records(specs, images, hip_device, seed=5)
    kfac = KFAC(net)
    kfac.launch_first = 16
    slow = []
    orig = KFAC._remember

    def counting(self, *a, **k):
        slow.append(1)
        return orig(self, *a, **k)
    KFAC._remember = counting
    try:
        per_pass, results = [], []
        for _ in range(4):
            n0 = len(slow)
            kfac.reset()
            for i in range(0, images, batch):
                for layer, (a, g) in zip(layers, recs):
                    kfac.record[layer] = [a[i:i + batch], g[i:i + batch]]
                kfac.update(batch_size=min(batch, images - i))
            kfac.invert(0.2 ** 2, 200)
            per_pass.append(len(slow) - n0)
            results.append([t.clone() for m in layers for t in list(kfac.state[m]) + list(kfac.inv_state[m])])
    finally:
        KFAC._remember = orig
    assert per_pass[2:] == [0, 0], per_pass
    for later in results[1:]:
        for a, b in zip(results[0], later):
            assert torch.equal(a, b)
