"""Control for the exit-time SIGSEGV seen under `rocprofv3 --pmc`:
plain torch GPU work of about the eig pass's length, with libkfac_hip.so never
loaded, so a crash here is the profiler's / runtime's teardown, not the library's."""
import json
import time

import torch

dev = torch.device("cuda:0")
x = torch.randn(4096, 4096, device=dev, dtype=torch.float64)
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(20):
    y = x @ x
    x = y / y.abs().max()
torch.cuda.synchronize()
print(json.dumps({"control_ms": (time.perf_counter() - t0) * 1e3, "kfac_loaded": False}), flush=True)
