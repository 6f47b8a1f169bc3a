"""CPU: the drop-in's host-side contract (models/curvatures.py:38-65, 295-398 semantics)."""
import numpy as np
import pytest
import torch
import torch.nn as nn

import host_double
from oracle import kfac_oracle as O


def mlp():
    torch.manual_seed(0)
    return nn.Sequential(nn.Linear(6, 5), nn.ReLU(), nn.Linear(5, 3))


def test_layer_type_selection():
    from bnn_kfac_amd.curvatures import KFAC
    net = mlp()
    assert KFAC(net, 'Linear').layer_types == ['Linear']
    assert KFAC(net, []).layer_types == ['Linear', 'Conv2d', 'MultiheadAttention']
    assert KFAC(net, None).layer_types == ['Linear', 'Conv2d', 'MultiheadAttention']
    with pytest.raises(TypeError):
        KFAC(net, 5)
    with pytest.raises(AssertionError):
        KFAC(net, ['Dense'])
    k = KFAC(net, ['Conv2d'])
    assert k.record == {} and k.hooks == []


def test_multihead_attention_not_implemented():
    from bnn_kfac_amd.curvatures import KFAC
    net = nn.Sequential(nn.MultiheadAttention(8, 2))
    with pytest.raises(NotImplementedError):
        KFAC(net)
    KFAC(net, 'Linear')  # excluding the type skips it (its out_proj is a Linear subclass)


def test_hooks_record_input_and_scaled_grad_output():
    from bnn_kfac_amd.curvatures import KFAC
    net = mlp()
    kfac = KFAC(net)
    x = torch.rand(4, 6)
    out = net(x)
    out.sum().div(4).backward()
    a, g = kfac.record[net[0]]
    assert a is x  # reference keeps the input itself (curvatures.py:319-320)
    # grad_output * batch (curvatures.py:322-323): d(sum/4)/d(out) * 4 = 1 for the last layer
    assert torch.allclose(kfac.record[net[2]][1], torch.ones(4, 3))
    assert g.shape == (4, 5)


def test_invert_requires_state():
    from bnn_kfac_amd.curvatures import KFAC
    with pytest.raises(AssertionError, match="State dict is empty"):
        KFAC(mlp()).invert(1.0, 1.0)


def test_no_cpu_fallback():
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import KFAC
    net = mlp()
    kfac = KFAC(net)
    net(torch.rand(3, 6)).sum().backward()
    with pytest.raises(N.NativeError, match="no CPU fallback"):
        kfac.update(3)


def test_damping_argument_handling():
    from bnn_kfac_amd.curvatures import KFAC
    kfac = KFAC(mlp())
    kfac.state = {1: None, 2: None}
    assert kfac._damping(0.04, 200) == [(0.04, 200.0), (0.04, 200.0)]
    assert kfac._damping([1, 2], [3, 4]) == [(1, 3), (2, 4)]
    with pytest.raises(AssertionError):
        kfac._damping([1], [3, 4])
    with pytest.raises(TypeError):  # mixed list/scalar: float(list) (curvatures.py:378)
        kfac._damping([1, 2], 3.0)


def test_update_host_logic_with_double(monkeypatch):
    """Packed buffer, per-batch alpha, first-assign / then-accumulate, modules() order."""
    from bnn_kfac_amd.curvatures import KFAC
    host_double.install(monkeypatch)
    net = mlp()
    kfac = KFAC(net)
    ref = O.OracleKFAC(np.float64)
    rng = np.random.default_rng(0)
    for B in (7, 7, 3):
        a1 = rng.random((B, 6), dtype=np.float32)
        g1 = rng.standard_normal((B, 5)).astype(np.float32)
        a2 = rng.random((B, 5), dtype=np.float32)
        g2 = rng.standard_normal((B, 3)).astype(np.float32)
        kfac.record[net[0]] = [torch.from_numpy(a1), torch.from_numpy(g1)]
        kfac.record[net[2]] = [torch.from_numpy(a2), torch.from_numpy(g2)]
        kfac.update(B)
        ref.update_linear("l0", a1, g1, True)
        ref.update_linear("l1", a2, g2, True)
    assert list(kfac.state) == [net[0], net[2]]
    A0, G0 = kfac.state[net[0]]
    assert A0.data_ptr() == kfac._packed.data_ptr()  # first factor at the buffer start
    np.testing.assert_allclose(A0.numpy(), ref.state["l0"][0], rtol=1e-5)
    np.testing.assert_allclose(G0.numpy(), ref.state["l0"][1], rtol=1e-5)
    np.testing.assert_allclose(kfac.state[net[2]][0].numpy(), ref.state["l1"][0], rtol=1e-5)
    # reset() alternates two packed buffers (an overlapped inversion reads one while
    # the next pass accumulates into the other); the second is allocated lazily
    first = kfac._packed
    kfac.reset()
    assert kfac.state == {} and kfac._packed is None and kfac._alt_packed is first
    kfac.record[net[0]] = [torch.from_numpy(a1), torch.from_numpy(g1)]
    kfac.record[net[2]] = [torch.from_numpy(a2), torch.from_numpy(g2)]
    kfac.update(B)
    second = kfac._packed
    assert second is not None and second.data_ptr() != first.data_ptr()
    kfac.reset()
    assert kfac._packed is first and kfac._alt_packed is second
    kfac.double_buffer = False
    kfac.reset()
    assert kfac._packed is first


def test_deferred_reduce_host_logic(monkeypatch):
    """Deferred reduction: a pass of updates keeps partials in accumulators and
    reduces ONCE when `state` is read; an update after that read starts a new cycle
    that adds to the factors (flush beta 1); results equal the immediate path."""
    from bnn_kfac_amd.curvatures import KFAC
    host_double.install(monkeypatch)
    host_double.FLUSHES.clear()
    rng = np.random.default_rng(3)
    batches = []
    for B in (8, 8, 5, 8):
        batches.append([torch.tensor(rng.random((B, 6), dtype=np.float32)),
                        torch.tensor(rng.standard_normal((B, 5)).astype(np.float32)),
                        torch.tensor(rng.random((B, 5), dtype=np.float32)),
                        torch.tensor(rng.standard_normal((B, 3)).astype(np.float32))])

    def run(defer, read_after):
        net = mlp()
        kfac = KFAC(net)
        kfac.defer_reduce = defer
        for i, (a1, g1, a2, g2) in enumerate(batches):
            kfac.record[net[0]] = [a1, g1]
            kfac.record[net[2]] = [a2, g2]
            kfac.update(a1.shape[0])
            if i == read_after:
                _ = kfac.state  # completes the pending reduction
        return [t.clone().numpy() for pair in kfac.state.values() for t in pair]

    want = run(False, -1)
    assert host_double.FLUSHES == []
    got = run(True, -1)
    assert host_double.FLUSHES == [4]  # one flush (4 factors) for 4 updates
    for g, w in zip(got, want):
        np.testing.assert_allclose(g, w, rtol=1e-6)
    host_double.FLUSHES.clear()
    got = run(True, 1)
    assert host_double.FLUSHES == [4, 4]  # read mid-pass, then the rest of the pass
    for g, w in zip(got, want):
        np.testing.assert_allclose(g, w, rtol=1e-6)


def test_invert_reduces_pass_on_side_stream(monkeypatch):
    """invert() of a pass whose reduction is deferred issues that reduce on the
    inversion's side stream (reduce_on_side), the cycles' accumulators alternate between
    two buffers, `state` afterwards holds the reduced factors; an invert() that raises
    before the side stream takes the reduce (bad damping) reduces on the caller's
    stream instead, and off (reduce_on_side False) the reduce stays there."""
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import KFAC
    host_double.install(monkeypatch)
    monkeypatch.setattr(N, "RawEvent", host_double.HostRawEvent)
    monkeypatch.setattr(N, "invert_pipelined", host_double.fake_invert_pipelined)
    monkeypatch.setattr(N, "stream_handle", lambda device: 0)

    class Side:
        cuda_stream = 7

    rng = np.random.default_rng(5)
    net = mlp()
    kfac = KFAC(net)
    kfac._inv_streams[None] = Side()  # (a single side stream set by hand; CPU device index)
    kfac._pinned_host = lambda n: torch.empty(n, dtype=torch.int32)
    accs = []
    for cycle in range(4):
        host_double.FLUSH_STREAMS.clear()
        kfac.reset()
        ref = O.OracleKFAC(np.float64)
        for B in (6, 4):
            a1 = rng.random((B, 6), dtype=np.float32)
            g1 = rng.standard_normal((B, 5)).astype(np.float32)
            a2 = rng.random((B, 5), dtype=np.float32)
            g2 = rng.standard_normal((B, 3)).astype(np.float32)
            kfac.record[net[0]] = [torch.from_numpy(a1), torch.from_numpy(g1)]
            kfac.record[net[2]] = [torch.from_numpy(a2), torch.from_numpy(g2)]
            kfac.update(B)
            ref.update_linear("l0", a1, g1, True)
            ref.update_linear("l1", a2, g2, True)
        accs.append(kfac._acc_map and min(a for a, _, _ in kfac._acc_map.values()))
        if cycle == 2:
            with pytest.raises(AssertionError):
                kfac.invert([0.04], [200.0, 200.0])  # damping list of the wrong length
            assert host_double.FLUSH_STREAMS == [None]  # reduced on the caller's stream
        else:
            kfac.invert(0.04, 200)
            assert host_double.FLUSH_STREAMS == [7]  # the reduce went to the side stream
        for m, name in ((net[0], "l0"), (net[2], "l1")):
            for got, want in zip(kfac.state[m], ref.state[name]):
                np.testing.assert_allclose(got.numpy(), want, rtol=1e-5)
            if cycle != 2:
                for L, F in zip(kfac.inv_state[m], kfac.state[m]):
                    np.testing.assert_allclose(L.numpy(), O.invert_factor(F.numpy().astype(np.float64), 0.04, 200),
                                               rtol=1e-4, atol=1e-6)
    # accumulators alternate after a side reduce (cycles 0, 1: two buffers), and a
    # cycle reduced on the caller's stream (2) leaves the turn where it was
    assert accs[0] != accs[1] and accs[2] == accs[0] and accs[3] == accs[0]
    host_double.FLUSH_STREAMS.clear()
    kfac.reduce_on_side = False
    kfac.reset()
    kfac.record[net[0]] = [torch.from_numpy(a1), torch.from_numpy(g1)]
    kfac.record[net[2]] = [torch.from_numpy(a2), torch.from_numpy(g2)]
    kfac.update(B)
    kfac.invert(0.04, 200)
    assert host_double.FLUSH_STREAMS == [None]


def test_queued_updates_merge_into_multibatch_jobs(monkeypatch):
    """update() queues; consecutive batches with matching operands become ONE
    multi-batch job per factor (K walks every queued batch), a batch of another
    shape starts a new group, `defer_batches` caps the queue, and the factors equal
    the one-launch-per-update path."""
    from bnn_kfac_amd.curvatures import KFAC
    host_double.install(monkeypatch)
    rng = np.random.default_rng(5)
    sizes = (8, 8, 8, 5, 8, 8)
    # torch.tensor copies into the CPU allocator's 64-byte-aligned blocks: equal
    # base alignment, as device allocations have (batches merge only then)
    batches = [[torch.tensor(rng.random((B, 6), dtype=np.float32)),
                torch.tensor(rng.standard_normal((B, 5)).astype(np.float32)),
                torch.tensor(rng.random((B, 5), dtype=np.float32)),
                torch.tensor(rng.standard_normal((B, 3)).astype(np.float32))]
               for B in sizes]

    def run(defer_reduce, defer_batches=64, defer_bytes=256 << 20, launch_first=1, merge=True):
        host_double.UPDATES.clear()
        net = mlp()
        kfac = KFAC(net)
        kfac.merge_launches = merge
        kfac.defer_reduce, kfac.defer_batches = defer_reduce, defer_batches
        kfac.defer_bytes = defer_bytes
        kfac.launch_first = launch_first
        for a1, g1, a2, g2 in batches:
            kfac.record[net[0]] = [a1, g1]
            kfac.record[net[2]] = [a2, g2]
            kfac.update(a1.shape[0])
        factors = [t.clone().numpy() for pair in kfac.state.values() for t in pair]
        return factors, [list(u) for u in host_double.UPDATES]

    want, launches = run(False)
    assert launches == [[1] * 4] * 6
    got, launches = run(True)  # launch sizes 1, 2, 4: [8] [8 8 | 5] [8 8]
    assert launches == [[1] * 4, [2] * 4, [1] * 4, [2] * 4]
    for g, w in zip(got, want):
        np.testing.assert_allclose(g, w, rtol=1e-6)
    got, launches = run(True, defer_batches=2)  # [8] [8 8] [5 8] [8]
    assert launches == [[1] * 4, [2] * 4, [1] * 4, [1] * 4, [1] * 4]
    for g, w in zip(got, want):
        np.testing.assert_allclose(g, w, rtol=1e-6)
    # a first launch of 16 queued updates: the whole pass is queued until the flush,
    # one multi-batch job per merge group, the short batch the ragged last batch of the
    # group before it (x.last_rows), all groups in ONE launch (each factor's two jobs on
    # their own accumulator slab ranges): [8 8 8 5* | 8 8]
    got, launches = run(True, launch_first=16)
    assert launches == [[4] * 4 + [2] * 4]
    for g, w in zip(got, want):
        np.testing.assert_allclose(g, w, rtol=1e-6)
    # merge_launches off: one launch call per merge group
    got, launches = run(True, launch_first=16, merge=False)
    assert launches == [[4] * 4, [2] * 4]
    for g, w in zip(got, want):
        np.testing.assert_allclose(g, w, rtol=1e-6)
    # defer_bytes caps the records a queue holds: an 8-row update keeps 608 bytes,
    # a 5-row one 380 -> [8] [8] [8] [5 | 8] [8]
    got, launches = run(True, defer_bytes=600)
    assert launches == [[1] * 4] * 6
    for g, w in zip(got, want):
        np.testing.assert_allclose(g, w, rtol=1e-6)


def test_fast_path_across_cycles(monkeypatch):
    """Passes of full batches and a short last one, reset() between them (the bench's
    loop, double-buffered packed state): after one pass per packed buffer, no update
    takes the slow path any more -- the cycle's first update starts from the buffer's
    cached template (beta 0, state entries re-created), the short batch from this
    cycle's alternate template -- and every pass's factors equal the immediate path's."""
    from bnn_kfac_amd.curvatures import KFAC
    host_double.install(monkeypatch)
    rng = np.random.default_rng(11)
    sizes = (8, 8, 8, 5)
    batches = [[torch.tensor(rng.random((B, 6), dtype=np.float32)),
                torch.tensor(rng.standard_normal((B, 5)).astype(np.float32)),
                torch.tensor(rng.random((B, 5), dtype=np.float32)),
                torch.tensor(rng.standard_normal((B, 3)).astype(np.float32))]
               for B in sizes]
    net = mlp()
    ref = KFAC(net)
    ref.defer_reduce = False
    for a1, g1, a2, g2 in batches:
        ref.record[net[0]], ref.record[net[2]] = [a1, g1], [a2, g2]
        ref.update(a1.shape[0])
    want = [t.clone().numpy() for pair in ref.state.values() for t in pair]
    kfac = KFAC(net)
    kfac.launch_first = 16
    slow = []
    orig = KFAC._remember
    monkeypatch.setattr(KFAC, "_remember", lambda self, *a, **k: (slow.append(1), orig(self, *a, **k))[1])
    per_pass = []
    for p in range(5):
        kfac.reset()
        n0 = len(slow)
        for a1, g1, a2, g2 in batches:
            kfac.record[net[0]], kfac.record[net[2]] = [a1, g1], [a2, g2]
            kfac.update(a1.shape[0])
        per_pass.append(len(slow) - n0)
        got = [t.clone().numpy() for pair in kfac.state.values() for t in pair]
        assert list(kfac.state) == [net[0], net[2]]  # modules() order
        for g, w in zip(got, want):
            np.testing.assert_allclose(g, w, rtol=1e-6)
    assert per_pass == [2, 2, 0, 0, 0]
    # a record of a new shape still takes the slow path (and is cached from then on)
    kfac.reset()
    a1, g1, a2, g2 = [t[:3] for t in batches[0]]
    kfac.record[net[0]], kfac.record[net[2]] = [a1, g1], [a2, g2]
    n0 = len(slow)
    kfac.update(3)
    assert len(slow) == n0 + 1


def test_queued_record_modified_in_place_raises(monkeypatch):
    from bnn_kfac_amd.curvatures import KFAC
    host_double.install(monkeypatch)
    net = mlp()
    kfac = KFAC(net)
    for _ in range(2):  # the first update launches at once, the second is queued
        a1 = torch.rand(4, 6)
        kfac.record[net[0]] = [a1, torch.randn(4, 5)]
        kfac.record[net[2]] = [torch.rand(4, 5), torch.randn(4, 3)]
        kfac.update(4)
    a1.mul_(2.0)
    with pytest.raises(RuntimeError, match="modified in place"):
        _ = kfac.state


def test_save_load_roundtrip(tmp_path):
    from bnn_kfac_amd.curvatures import KFAC
    net = mlp()
    kfac = KFAC(net)
    kfac.state = {net[0]: [torch.eye(7), torch.eye(5)], net[2]: [torch.eye(6), torch.eye(3)]}
    kfac.inv_state = {net[0]: (torch.eye(7) * 2, torch.eye(5) * 2)}
    fn = str(tmp_path / "kfac.pt")
    kfac.save(fn)
    other = KFAC(mlp())
    other.load(fn)
    assert [type(m).__name__ for m in other.state] == ["Linear", "Linear"]
    assert torch.equal(other.state[other.model[0]][0], torch.eye(7))
    assert torch.equal(other.inv_state[other.model[0]][1], torch.eye(5) * 2)
    for p, q in zip(net.parameters(), other.model.parameters()):
        assert torch.equal(p, q)


def test_kron_doctest():
    import doctest

    from bnn_kfac_amd import utilities
    res = doctest.testmod(utilities)
    assert res.failed == 0 and res.attempted >= 1


def test_variance_helpers():
    from bnn_kfac_amd.variance import argmax_grad_outputs, entropy_bits
    p = torch.tensor([[0.1, 0.7, 0.2], [0.5, 0.2, 0.3]])
    go = argmax_grad_outputs(p)
    # classification_ll_block.py:119-121: every argmax column set in EVERY row
    assert torch.equal(go, torch.tensor([[1., 1., 0.], [1., 1., 0.]]))
    assert abs(entropy_bits(1.0) - 0.5 * np.log2(2 * np.e * np.pi)) < 1e-12


def _host_chol_inverse(R, shifts):
    """Host test double of INF._chol_inverse (kfac_invert on the device)."""
    import torch
    eye = torch.eye(R.shape[0], dtype=R.dtype)
    return [torch.linalg.inv(torch.linalg.cholesky(R + t * eye)) for t in shifts]


def test_inf_host_algebra_matches_literal_oracle():
    """INF's tensor restatements (curvatures.py:614-682: index arithmetic, the per-row
    kron loop; :548-580 the pre-sample after the Gram matrix) against the literal
    loop/kron oracle.  These are torch algebra on whatever device the tensors live;
    here CPU, no kernel call.  The Gram matrix itself is device-only."""
    import numpy as np
    import torch
    import pytest
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import INF
    from oracle import kfac_oracle as O
    rng = np.random.default_rng(3)
    U_A = np.linalg.qr(rng.standard_normal((9, 9)))[0]
    U_G = np.linalg.qr(rng.standard_normal((4, 4)))[0]
    lam = rng.random(36) + 0.1
    for rank in (1, 5, 17, 36, 100):
        a, b, lr = INF._dim_reduction(*(torch.from_numpy(x) for x in (U_A, U_G, lam)), rank)
        wa, wb, wl = O.inf_dim_reduction(U_A, U_G, lam, rank)
        np.testing.assert_array_equal(a.numpy(), wa)
        np.testing.assert_array_equal(b.numpy(), wb)
        np.testing.assert_array_equal(lr.numpy(), wl)
        d = INF._diagonal_accumulator(a, b, lr).numpy()
        np.testing.assert_allclose(d, O.inf_diagonal_accumulator(wa, wb, wl), rtol=1e-12)
        sig = np.sqrt(200 * np.asarray(wl))
        c = 1.0 / np.sqrt(200 * rng.random(36) + 0.04)
        # the pre-sample's linear algebra after the Gram matrix (the Gram itself is
        # kfac_kron_gram on the device: pre_sampler has no host path)
        Vs = c[:, None] * np.kron(wa, wb) * sig[None, :]
        P = INF._pre_sample_from_gram(torch.from_numpy(Vs.T @ Vs), torch.from_numpy(sig),
                                      chol_inverse=_host_chol_inverse).numpy()
        np.testing.assert_allclose(P, O.inf_pre_sampler(wa, wb, sig, c), rtol=1e-8, atol=1e-12)
        with pytest.raises(N.NativeError):
            INF.pre_sampler(a, b, torch.from_numpy(sig), torch.from_numpy(c))


def test_sample_has_no_cpu_fallback():
    """KFAC.sample / sample_and_replace go through kfac_sample only: host tensors raise."""
    import pytest
    import torch
    from bnn_kfac_amd import _native as N
    from bnn_kfac_amd.curvatures import KFAC
    net = torch.nn.Sequential(torch.nn.Linear(6, 3))
    kfac = KFAC(net)
    kfac.inv_state = {net[0]: (torch.eye(7), torch.eye(3))}
    with pytest.raises(N.NativeError):
        kfac.sample(net[0])
    with pytest.raises(N.NativeError):
        kfac.sample_and_replace()


def test_distributed_world1_state_read_completes_pass(monkeypatch, tmp_path):
    """DistributedKFAC at world 1 (no process group): `update(); kfac.state` holds the
    whole pass, as with KFAC -- the pending pass needs no collective, so the read sums
    it in (was: {} with a warning).  save() after it writes that state."""
    import warnings
    from bnn_kfac_amd.distributed import DistributedKFAC
    host_double.install(monkeypatch)
    net = mlp()
    kfac = DistributedKFAC(net)
    assert kfac.world == 1 and not kfac._collective()
    ref = O.OracleKFAC(np.float64)
    rng = np.random.default_rng(3)
    for p in range(2):
        for B in (7, 4):
            a1 = rng.random((B, 6), dtype=np.float32)
            g1 = rng.standard_normal((B, 5)).astype(np.float32)
            a2 = rng.random((B, 5), dtype=np.float32)
            g2 = rng.standard_normal((B, 3)).astype(np.float32)
            kfac.record[net[0]] = [torch.from_numpy(a1), torch.from_numpy(g1)]
            kfac.record[net[2]] = [torch.from_numpy(a2), torch.from_numpy(g2)]
            kfac.update(B)
            ref.update_linear("l0", a1, g1, True)
            ref.update_linear("l1", a2, g2, True)
        with warnings.catch_warnings():
            warnings.simplefilter("error")  # no "not all-reduced" warning at world 1
            st = kfac.state
        assert not kfac._pending
        np.testing.assert_allclose(st[net[0]][0].numpy(), ref.state["l0"][0], rtol=1e-5)
        np.testing.assert_allclose(st[net[2]][1].numpy(), ref.state["l1"][1], rtol=1e-5)
    kfac.save(str(tmp_path / "w1.pt"))  # (inv_state empty: nothing inverted)
    blob = torch.load(str(tmp_path / "w1.pt"), weights_only=True)
    np.testing.assert_allclose(blob["state"]["0"][0].numpy(), ref.state["l0"][0], rtol=1e-5)


def test_distributed_save_refused_while_pass_pending(monkeypatch, tmp_path):
    """With a collective to run (world > 1, modelled by always_reduce), save() refuses
    while this rank's pass is not all-reduced instead of leaving it out silently."""
    from bnn_kfac_amd.distributed import DistributedKFAC
    host_double.install(monkeypatch)
    net = mlp()
    kfac = DistributedKFAC(net)
    kfac.always_reduce = True
    rng = np.random.default_rng(4)
    kfac.record[net[0]] = [torch.from_numpy(rng.random((3, 6), dtype=np.float32)),
                           torch.from_numpy(rng.standard_normal((3, 5)).astype(np.float32))]
    kfac.record[net[2]] = [torch.from_numpy(rng.random((3, 5), dtype=np.float32)),
                           torch.from_numpy(rng.standard_normal((3, 3)).astype(np.float32))]
    kfac.update(3)
    with pytest.raises(RuntimeError, match="not all-reduced"):
        kfac.save(str(tmp_path / "x.pt"))
