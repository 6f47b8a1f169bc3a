"""Time KFAC.sample_and_replace (kfac_sample, one launch pair over all layers) against
the reference's op sequence (curvatures.py:117-129 + 400-405 + 68-82: per layer randn,
two matmuls, transpose, bias/weight adds) run with torch on the same GPU and on the
host CPU.  Writes gpurun_out/sample.json."""
import json
import os
import sys
import time

import torch
import torch.nn as nn

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bnn_kfac_amd.curvatures import KFAC  # noqa: E402


def ref_sample_and_replace(net, inv, state):
    """The reference's op sequence (models/curvatures.py:117-129, 400-405, 68-82)."""
    net.load_state_dict(state)
    for m in net.modules():
        if isinstance(m, (nn.Linear, nn.Conv2d)):
            first, second = inv[m]
            z = torch.randn(first.size(0), second.size(0), device=first.device)
            s = (first @ z @ second.t()).t()
            if m.bias is not None:
                m.bias.data.add_(s[:, -1].contiguous().view(*m.bias.shape))
                s = s[:, :-1]
            m.weight.data.add_(s.contiguous().view(*m.weight.shape))


def tril_chol(n, dev):
    X = torch.randn(n, n + 8, device=dev)
    return torch.linalg.cholesky(X @ X.t() / n + torch.eye(n, device=dev))


def timeit(fn, sync, reps):
    for _ in range(3):
        fn()
    sync()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    sync()
    return (time.perf_counter() - t) / reps


def main():
    dev = torch.device("cuda:0")
    out = {}
    for name, widths in (("mlp", [784, 128, 10]), ("wide", [784, 4096, 4096, 10])):
        torch.manual_seed(0)
        layers = [nn.Linear(a, b) for a, b in zip(widths[:-1], widths[1:])]
        net = nn.Sequential(*layers).to(dev)
        kfac = KFAC(net)
        inv = {m: (tril_chol(m.in_features + 1, dev), tril_chol(m.out_features, dev)) for m in layers}
        kfac.inv_state = inv
        state = {k: v.clone() for k, v in net.state_dict().items()}
        sync = torch.cuda.synchronize
        reps = 50 if name == "mlp" else 5
        t_hip = timeit(kfac.sample_and_replace, sync, reps)
        t_torch = timeit(lambda: ref_sample_and_replace(net, inv, state), sync, reps)
        net_c = nn.Sequential(*[nn.Linear(a, b) for a, b in zip(widths[:-1], widths[1:])])
        inv_c = {mc: tuple(t.cpu() for t in inv[m]) for mc, m in zip(net_c, layers)}
        state_c = net_c.state_dict()
        t_cpu = timeit(lambda: ref_sample_and_replace(net_c, inv_c, state_c), lambda: None,
                       20 if name == "mlp" else 1)
        flops = sum(2 * (m.in_features + 1) ** 2 * m.out_features / 2 +
                    2 * (m.in_features + 1) * m.out_features ** 2 / 2 for m in layers)
        out[name] = dict(kfac_sample_ms=t_hip * 1e3, torch_gpu_ref_ms=t_torch * 1e3,
                         cpu_ref_ms=t_cpu * 1e3, cpu_threads=torch.get_num_threads(),
                         triangular_gflop=flops / 1e9, kfac_sample_tflops=flops / t_hip / 1e12)
        print(name, json.dumps(out[name]), flush=True)
    os.makedirs("gpurun_out", exist_ok=True)
    with open("gpurun_out/sample.json", "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
