"""GPU, world_size 2 on one device (gloo carries the collective; RCCL cannot put two
ranks on one GPU): the data-parallel factor pass with the real HIP kernels reproduces
single-device KFAC — same factors (one packed all-reduce per pass) and the same
inverse Cholesky factors — over two passes with an uneven last batch."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

SIZES = (512, 512, 300)  # global batches; the last one splits unevenly over 2 ranks


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _data():
    rng = np.random.default_rng(7)
    out = []
    for gb in SIZES:
        out.append((rng.random((gb, 784), dtype=np.float32),
                    rng.standard_normal((gb, 128)).astype(np.float32),
                    rng.random((gb, 128), dtype=np.float32),
                    rng.standard_normal((gb, 10)).astype(np.float32)))
    return out


def _net(dev):
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Linear(784, 128), torch.nn.ReLU(),
                               torch.nn.Linear(128, 10)).to(dev)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank),
                      WORLD_SIZE=str(world))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from bnn_kfac_amd.distributed import DistributedKFAC
        dev = torch.device("cuda:0")
        net = _net(dev)
        kfac = DistributedKFAC(net)
        for p in range(2):
            kfac.reset()
            for a1, g1, a2, g2 in _data():
                gb = a1.shape[0]
                cut = [0, gb // 2 + 37, gb][rank:rank + 2]  # uneven shards
                sl = slice(*cut)
                kfac.record[net[0]] = [torch.from_numpy(a1[sl]).to(dev), torch.from_numpy(g1[sl]).to(dev)]
                kfac.record[net[2]] = [torch.from_numpy(a2[sl]).to(dev), torch.from_numpy(g2[sl]).to(dev)]
                kfac.update(cut[1] - cut[0], global_batch_size=gb)
            kfac.invert(0.04, 200)
        st = [t.cpu().numpy() for pair in kfac.state.values() for t in pair]
        inv = [t.cpu().numpy() for pair in kfac.inv_state.values() for t in pair]
        q.put((rank, st, inv))
    finally:
        dist.destroy_process_group()


def test_two_ranks_match_single_device(hip_device):
    from bnn_kfac_amd.curvatures import KFAC
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    results = sorted([q.get(timeout=300) for _ in procs], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    net = _net(hip_device)
    kfac = KFAC(net)
    for a1, g1, a2, g2 in _data():
        kfac.record[net[0]] = [torch.from_numpy(a1).to(hip_device), torch.from_numpy(g1).to(hip_device)]
        kfac.record[net[2]] = [torch.from_numpy(a2).to(hip_device), torch.from_numpy(g2).to(hip_device)]
        kfac.update(a1.shape[0])
    kfac.invert(0.04, 200)
    want_st = [t.cpu().numpy() for pair in kfac.state.values() for t in pair]
    want_inv = [t.cpu().numpy() for pair in kfac.inv_state.values() for t in pair]
    for rank, st, inv in results:
        for g, w in zip(st, want_st):
            np.testing.assert_allclose(g, w, rtol=1e-5, atol=1e-5 * np.abs(w).max())
        # replicated inversion of the reduced factors: the sharded sums differ from the
        # single-device ones in the last bits, which the inversion amplifies by cond(R)
        # (~1e5 here) -> normwise 1e-4 (the north-star tolerance)
        for g, w in zip(inv, want_inv):
            np.testing.assert_allclose(g, w, rtol=0, atol=1e-4 * np.abs(w).max())
    np.testing.assert_array_equal(results[0][2][0], results[1][2][0])  # ranks agree exactly
