"""GPU parity at BASELINE C2's stated config, run exactly as bench.py's headline loop
runs it: the MLP 784-128-10 over one MNIST-sized pass of 60,000 images at batch
4,096 (14 full batches + a 2,656-row last batch), KFAC.launch_first 16 (the pass's
queued updates go out at the flush as ONE multi-batch x3 launch: the full batches and
the short last batch as its ragged last segment, with the planner's K-split plan -- f
full-tile K-splits plus the thin-row pair units' extra K-splits), deferred reduction,
double-buffered state, eager_verdict False and invert(0.04, 200) pipelined: pass 2 is
queued behind inversion 1 on its side stream before any verdict is read.

Every A / G of pass 2 against the fp64 oracle (models/curvatures.py:345-363:
O.linear_factor_A / O.grad_factor, sum of per-batch means) at rtol 1e-5, and every L
against O.invert_factor (curvatures.py:381-398) on the device's own factor within 1e-4
of max|L|.  Pass 1's L factors (read after pass 2 was queued) must be bit-identical to
pass 2's: same records, deterministic kernels.
"""
import numpy as np
import pytest
import torch

import bench
from oracle import kfac_oracle as O

pytestmark = pytest.mark.gpu

IMAGES, BATCH = 60000, 4096


def test_mlp_c2_bench_pass_pipelined_vs_fp64_oracle(hip_device):
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import KFAC
    assert IMAGES % BATCH == 2656
    specs = bench.CONFIGS["mlp"]
    net = bench.build_model("mlp", hip_device)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(specs, IMAGES, hip_device, seed=2024)
    kfac = KFAC(net)
    kfac.eager_verdict = False
    kfac.launch_first = 16
    starts = list(range(0, IMAGES, BATCH))
    launches = []
    orig = N.factor_update

    def counting(jobs, device):
        launches.append([(j.x.rows * (j.nseg - 1) + (j.x.last_rows or j.x.rows)) if j.nseg > 1
                         else j.x.rows for j in jobs])
        return orig(jobs, device)

    def one_pass():
        kfac.reset()
        for i in starts:  # bench.py one_pass
            for layer, (a, g) in zip(layers, recs):
                kfac.record[layer] = [a[i:i + BATCH], g[i:i + BATCH]]
            kfac.update(batch_size=min(BATCH, IMAGES - i))
        kfac.invert(*bench.DAMPING)

    N.factor_update = counting
    try:
        one_pass()
        first = kfac._inv_pending  # pass 1's L factors, verdict not read yet
        assert first is not None and first.on_side
        L1 = [t for t in first.outs]
        one_pass()  # queued behind inversion 1, double-buffered state
        inv = kfac.inv_state  # settles both verdicts
    finally:
        N.factor_update = orig
    # the headline's launch structure: ONE launch per pass, every factor one multi-batch
    # job over the 14 full batches and the 2,656-row last one (x.last_rows)
    assert launches == [[IMAGES] * 4] * 2, launches
    state = [[t.cpu().numpy() for t in kfac.state[m]] for m in layers]
    Ls = [[t.cpu().numpy() for t in inv[m]] for m in layers]
    for a, b in zip(L1, [t for m in layers for t in inv[m]]):
        assert torch.equal(a, b)
    recs_cpu = [(a.cpu().numpy(), g.cpu().numpy()) for a, g in recs]
    del recs
    for li, (l, (x, g)) in enumerate(zip(specs, recs_cpu)):
        wA = sum(O.linear_factor_A(x[i:i + BATCH], True, np.float64) for i in starts)
        wG = sum(O.grad_factor(g[i:i + BATCH], np.float64) for i in starts)
        A, G = state[li]
        for name, got, ref in (("A", A, wA), ("G", G, wG)):
            np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max(),
                                       err_msg=f"layer {li} {name}")
        for name, F, L in (("L_A", A, Ls[li][0]), ("L_G", G, Ls[li][1])):
            ref = O.invert_factor(F.astype(np.float64), *bench.DAMPING)
            np.testing.assert_allclose(L, ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max(),
                                       err_msg=f"layer {li} {name}")
            assert np.all(np.triu(L, 1) == 0)
