"""CPU, world 2 over gloo: bench.verify_parity, the N > 1 self-check that runs after
the timed region of `bench.py --gpus N` (the sharded pass + all-reduce vs rank 0's
single-device recompute of the same global batches, models/curvatures.py:359-363).
The device kernels are the host test double (tests/host_double.py); what runs is
the bench's verification logic and the product's data-parallel host code.  Two
negative cases show that the check can fail: records regenerated from the wrong
seed (checksum mismatch) and an all-reduce that is skipped (factor mismatch)."""
import os
import socket
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q, scenario):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        sys.path.insert(0, ROOT)
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import bench
        import host_double
        from bnn_kfac_amd import _native as N
        from bnn_kfac_amd.curvatures import KFAC
        from bnn_kfac_amd.distributed import DistributedKFAC
        host_double.install_distributed()
        torch.manual_seed(0)
        net = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
        specs = [bench.Layer("linear", 6, 5), bench.Layer("linear", 5, 3)]
        dev = torch.device("cpu")
        images, batch = 20, 8
        recs = bench.synthetic_records(specs, images, dev, seed=1234 + rank)
        kfac = DistributedKFAC(net)
        host_double.install_distributed(kfac)
        host_double.install_cuda_stubs([kfac])
        if scenario == "no_allreduce":
            N.tri_unpack = lambda jobs, packed, mode: None  # the reduced sums never land

        def ref_factory(model):
            ref = KFAC(model)
            host_double.install_cuda_stubs([ref])
            return ref
        seed0 = 999 if scenario == "wrong_seed" else 1234
        out = bench.verify_parity(kfac, net, specs, recs, batch, images, world, rank, dev,
                                  sync=lambda: None, nbatches=3, seed0=seed0,
                                  ref_factory=ref_factory)
        q.put((rank, out))
    except BaseException as e:  # report instead of leaving the parent waiting
        q.put((rank, repr(e)))
        raise
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("scenario,world", [("ok", 2), ("ok", 3), ("wrong_seed", 2),
                                            ("no_allreduce", 2)])
def test_verify_parity(scenario, world):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, scenario)) for r in range(world)]
    for p in procs:
        p.start()
    results = sorted([q.get(timeout=120) for _ in procs], key=lambda r: r[0])
    for _, out in results:
        assert isinstance(out, dict), out
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the verdict is broadcast: every rank reports the same one
    oks = {out["ok"] for _, out in results}
    assert len(oks) == 1
    detail = results[0][1]
    assert detail["batches"] == 3 and detail["rows_per_rank"] == 20
    if scenario == "ok":
        assert oks == {True}
        assert detail["records_checksum_match"] and detail["identical_L_all_ranks"]
        assert detail["max_rel_err_factors"] <= 1e-6 and detail["max_rel_err_L"] <= 1e-5
    elif scenario == "wrong_seed":
        assert oks == {False} and not detail["records_checksum_match"]
    else:  # each rank kept its own partial sums: wrong, and different on every rank
        assert oks == {False} and detail["max_rel_err_factors"] > 1e-2
        assert not detail["identical_L_all_ranks"]
