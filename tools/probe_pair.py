"""Time the MLP's grouped inversion (785, 128, 129, 10 factors, invert(0.04, 200)) alone
on the GPU: HIP-event time per call, mean of `reps`.  Written for the A/B of the
paired-step chain (commit d327996, KFAC_INV_PAIR, removed after it) and the
tasks-per-workgroup knob (KFAC_INV_TPW).  GPU only.

    python tools/probe_pair.py [reps]
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bnn_kfac_amd import _native as N  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 200
    dev = torch.device("cuda:0")
    rng = np.random.default_rng(0)
    Fs = []
    for n in (785, 128, 129, 10):
        x = rng.random((4 * n, n), dtype=np.float32)
        Fs.append(torch.from_numpy(x.T @ x / (4 * n)).to(dev))
    outs = [torch.empty_like(F) for F in Fs]
    jobs = [N.invert_job(F, o, 200 ** 0.5, 0.04 ** 0.5) for F, o in zip(Fs, outs)]
    for _ in range(20):
        N.invert(jobs, dev)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        info = N.invert(jobs, dev)
    e1.record()
    torch.cuda.synchronize()
    assert not info.cpu().any()
    print(f"pair={os.environ.get('KFAC_INV_PAIR', '0')} tpw={os.environ.get('KFAC_INV_TPW', 'default')}: "
          f"{e0.elapsed_time(e1) / reps * 1e3:.1f} us per grouped inversion (alone, back to back)")


if __name__ == "__main__":
    main()
