"""GPU parity at BASELINE C5's stated config, run exactly as bench.py runs it
(`other_configs.C5`): the wide MLP 784-4096-4096-10 over 16,384 images at batch 4,096,
KFAC.launch_first 16 with the library's 512 MiB records cap (each update holds 281 MB
of records, so a pass goes out as two kfac_factor_syrk3 launches of two batches each:
the n >= 2048 group, split into bf16x3 in the workgroup), deferred reduction,
double-buffered state, eager_verdict False and invert(0.04, 200) pipelined: the 4097^2
factors take the blocked 64-tile inversion (inv_panel / inv_inner / inv_bulk with the
look-ahead helper stream), and pass 2 is queued behind inversion 1 before any verdict
is read.

Every A / G of pass 2 against the fp64 oracle (models/curvatures.py:345-363:
O.linear_factor_A / O.grad_factor, sum of per-batch means) at rtol 1e-5, every L
against O.invert_factor (curvatures.py:381-398) on the device's own factor within 1e-4
of max|L|, and pass 1's L factors bit-identical to pass 2's.
"""
import numpy as np
import pytest
import torch

import bench
from oracle import kfac_oracle as O

pytestmark = pytest.mark.gpu

IMAGES, BATCH = 16384, 4096


def test_wide_c5_bench_pass_pipelined_vs_fp64_oracle(hip_device):
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import KFAC
    assert bench.SHAPES[("wide", 1)] == (BATCH, IMAGES)
    assert N.get_knob("KFAC_INV_LOOKAHEAD") == 1
    specs = bench.CONFIGS["wide"]
    net = bench.build_model("wide", hip_device)
    layers = [m for m in net.modules() if isinstance(m, torch.nn.Linear)]
    recs = bench.synthetic_records(specs, IMAGES, hip_device, seed=99)
    kfac = KFAC(net)
    kfac.eager_verdict = False
    kfac.launch_first = 16
    starts = list(range(0, IMAGES, BATCH))
    launches = []
    orig = N.factor_update

    def counting(jobs, device):
        launches.append([j.x.rows * max(j.nseg, 1) for j in jobs])
        return orig(jobs, device)

    def one_pass():
        kfac.reset()
        for i in starts:  # bench.py other_config's one_pass
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
    # the bench's launch structure: two launches of two batches per pass (records cap)
    assert launches == [[2 * BATCH] * 6] * 4, launches
    for a, b in zip(L1, [t for m in layers for t in inv[m]]):
        assert torch.equal(a, b)
    state = [[t.cpu().numpy() for t in kfac.state[m]] for m in layers]
    Ls = [[t.cpu().numpy() for t in inv[m]] for m in layers]
    del kfac, inv, L1, first
    recs_cpu = [(a.cpu().numpy(), g.cpu().numpy()) for a, g in recs]
    del recs
    torch.cuda.empty_cache()
    for li, (x, g) in enumerate(recs_cpu):
        wA = sum(O.linear_factor_A(x[i:i + BATCH], True, np.float64) for i in starts)
        wG = sum(O.grad_factor(g[i:i + BATCH], np.float64) for i in starts)
        A, G = state[li]
        for name, got, ref in (("A", A, wA), ("G", G, wG)):
            np.testing.assert_allclose(got, ref, rtol=1e-5, atol=1e-6 * np.abs(ref).max(),
                                       err_msg=f"layer {li} {name}")
        del wA, wG
        for name, F, L in (("L_A", A, Ls[li][0]), ("L_G", G, Ls[li][1])):
            ref = O.invert_factor(F.astype(np.float64), *bench.DAMPING)
            np.testing.assert_allclose(L, ref, rtol=1e-4, atol=1e-4 * np.abs(ref).max(),
                                       err_msg=f"layer {li} {name}")
            assert np.all(np.triu(L, 1) == 0)
