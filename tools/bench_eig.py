"""Time the device eigenvalue path (utilities.symeig) at the configs' factor sizes,
next to torch CPU eigvalsh (the reference's successor of torch.symeig)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, __import__("os").path.dirname(__import__("os").path.dirname(__file__)))
from bnn_kfac_amd.utilities import symeig  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    out = {}
    vecs = os.environ.get("EIG_VECS", "0") == "1"
    for n in [int(a) for a in sys.argv[1:]] or [129, 785, 4097]:
        rng = np.random.default_rng(n)
        X = rng.standard_normal((n, n)).astype(np.float32)
        F = torch.from_numpy(X @ X.T / n + 1e-3 * np.eye(n, dtype=np.float32))
        Fd = F.to(dev)
        symeig([Fd], eigenvectors=vecs)
        torch.cuda.synchronize()
        reps = 5 if not vecs else 2
        t0 = time.perf_counter()
        for _ in range(reps):
            ev = symeig([Fd], eigenvectors=vecs)[0][0]
        torch.cuda.synchronize()
        gpu_ms = (time.perf_counter() - t0) / reps * 1e3
        cpu_ms = err = None
        if os.environ.get("EIG_NO_CPU") != "1":  # (profiler passes: the device path only)
            t0 = time.perf_counter()
            want = torch.linalg.eigh(F.double())[0] if vecs else torch.linalg.eigvalsh(F.double())
            cpu_ms = (time.perf_counter() - t0) * 1e3
            err = float((ev.cpu() - want).abs().max() / want.abs().max())
        out[n] = {"gpu_ms": gpu_ms, "vectors": vecs, "cpu_fp64_ms": cpu_ms, "max_rel_err": err,
                  "cpu_threads": torch.get_num_threads()}
        print(json.dumps({n: out[n]}), flush=True)


if __name__ == "__main__":
    main()
    if os.environ.get("EIG_FAST_EXIT") == "1":
        # profiler passes: a process that ran a cooperative launch (eig_tridiag)
        # segfaults in exit() after rocprofv3 --pmc's tool finalization (not without
        # --pmc, not without the cooperative launch: tools/exit_probe.py, DESIGN.md
        # §3.4); leave without the exit handlers once the output is flushed
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
