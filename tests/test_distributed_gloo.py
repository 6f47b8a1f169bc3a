"""CPU, world_size 2 over gloo: the data-parallel factor pass reproduces the
single-device state (sum over global batches of per-global-batch means) with ONE
all-reduce of the packed buffer.  The device kernels are replaced by the host
test double (tests/host_double.py); the product's sharding/alpha/all-reduce
logic is what runs."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, result_q, scenario):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import sys
        sys.path.insert(0, os.path.dirname(__file__))
        import host_double
        from bnn_kfac_amd.distributed import DistributedKFAC
        host_double.install_distributed()
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
        kfac = DistributedKFAC(net)
        host_double.install_distributed(kfac)
        calls = {"n": 0}
        orig = dist.all_reduce

        def counting(*a, **k):
            calls["n"] += 1
            return orig(*a, **k)
        dist.all_reduce = counting
        rng = np.random.default_rng(42)  # same global data on every rank
        passes = 2 if scenario == "two_passes" else 1
        for _ in range(passes):
            for gb in (8, 8, 6):
                A1 = rng.random((gb, 6), dtype=np.float32)
                G1 = rng.standard_normal((gb, 5)).astype(np.float32)
                A2 = rng.random((gb, 5), dtype=np.float32)
                G2 = rng.standard_normal((gb, 3)).astype(np.float32)
                if scenario == "uneven":
                    cut = [0, 3, gb][rank:rank + 2]
                else:
                    cut = [rank * gb // world, (rank + 1) * gb // world]
                sl = slice(*cut)
                kfac.record[net[0]] = [torch.from_numpy(A1[sl]), torch.from_numpy(G1[sl])]
                kfac.record[net[2]] = [torch.from_numpy(A2[sl]), torch.from_numpy(G2[sl])]
                kfac.update(cut[1] - cut[0], global_batch_size=gb)
                if scenario == "state_read" and rank == 0:
                    # a rank-local read mid-pass (logging, rank-0 checkpoint): no
                    # collective, so it cannot hang the other ranks; it warns that the
                    # pending pass is not in the reduced state yet
                    import warnings
                    with warnings.catch_warnings(record=True) as w:
                        warnings.simplefilter("always")
                        assert kfac.state == {}
                    assert any("not all-reduced" in str(x.message) for x in w)
            kfac.allreduce()
        dist.all_reduce = orig
        out = [t.numpy().copy() for pair in kfac.state.values() for t in pair]
        inv = None
        if scenario in ("sharded", "sharded_singular", "sharded_singular_eager"):
            if scenario.startswith("sharded_singular"):
                # layer 1's G made indefinite: layers from the first failing one are
                # dropped and LinAlgError raised on every rank (curvatures.py:393-396)
                kfac.state[net[2]][1].fill_(-1.0)
            kfac.shard_inversion = True
            kfac.eager_verdict = scenario == "sharded_singular_eager"
            in_invert = True
            try:
                kfac.invert(0.04, 200)
                in_invert = False
                inv = [t.numpy().copy() for pair in kfac.inv_state.values() for t in pair]
            except np.linalg.LinAlgError:
                inv = ("LinAlgError", sorted(kfac._inv_state.keys(), key=id) == sorted([net[0]], key=id))
                if kfac.eager_verdict:  # eager: raised by invert() itself, as the reference
                    inv = inv + (in_invert,)
        result_q.put((rank, out, calls["n"], inv))
    finally:
        dist.destroy_process_group()


def _reference(scenario):
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(__file__)))
    from oracle import kfac_oracle as O
    ref = O.OracleKFAC(np.float64)
    rng = np.random.default_rng(42)
    passes = 2 if scenario == "two_passes" else 1
    for _ in range(passes):
        for gb in (8, 8, 6):
            A1 = rng.random((gb, 6), dtype=np.float32)
            G1 = rng.standard_normal((gb, 5)).astype(np.float32)
            A2 = rng.random((gb, 5), dtype=np.float32)
            G2 = rng.standard_normal((gb, 3)).astype(np.float32)
            ref.update_linear("l0", A1, G1, True)
            ref.update_linear("l1", A2, G2, True)
    return [ref.state["l0"][0], ref.state["l0"][1], ref.state["l1"][0], ref.state["l1"][1]]


@pytest.mark.parametrize("scenario,world", [("even", 2), ("uneven", 2), ("two_passes", 2),
                                            ("even", 4), ("state_read", 2), ("sharded", 2),
                                            ("sharded", 3), ("sharded_singular", 2),
                                            ("sharded_singular_eager", 2)])
def test_sharded_pass_matches_single_device(scenario, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, scenario)) for r in range(world)]
    for p in procs:
        p.start()
    results = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    want = _reference(scenario)
    for rank, got, n_allreduce, inv in results:
        # one packed all-reduce per pass (two_passes: two)
        assert n_allreduce == (2 if scenario == "two_passes" else 1)
        for g, w in zip(got, want):
            np.testing.assert_allclose(g, w, rtol=1e-5, atol=1e-6)
        if scenario == "sharded":
            # every rank holds every L factor (its own inverted, the rest gathered)
            from oracle import kfac_oracle as O
            for g, F in zip(inv, got):
                np.testing.assert_allclose(g, O.invert_factor(F.astype(np.float64), 0.04, 200),
                                           rtol=1e-5, atol=1e-6)
        if scenario == "sharded_singular":
            assert inv == ("LinAlgError", True)
        if scenario == "sharded_singular_eager":
            assert inv == ("LinAlgError", True, True)
