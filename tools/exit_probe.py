"""Exit-time SIGSEGV under `rocprofv3 --pmc`, bisected by what the
process did before exit:
  load    -- libkfac_hip.so loaded (ctypes), torch's HIP runtime up, no kfac launch
  factor  -- one kfac_factor_update (ordinary launches), kfac_release at exit
  eig     -- one kfac_syev at n = 4097 (cooperative launch), normal exit
  eig_os  -- the same, then os._exit(0) after flushing (no atexit / static destructors)
Before it exits the process writes /proc/self/maps to $EXIT_MAPS (if set), so the PCs
of a crash trace printed during exit can be mapped to a shared object + offset
(tools/exit_maps.py).
"""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bnn_kfac_amd import _native as N  # noqa: E402

mode = sys.argv[1]
dev = torch.device("cuda:0")
torch.zeros(1, device=dev)
N.lib()
if mode == "factor":
    x = torch.rand(4096, 784, device=dev)
    F = torch.empty(785, 785, device=dev)
    N.factor_update([N.factor_job(N.rowmajor_operand(x, True), F, 1.0 / 4096, 0.0)], dev)
elif mode.startswith("eig"):
    from bnn_kfac_amd.utilities import symeig
    n = 4097
    X = torch.randn(n, n, device=dev)
    F = X @ X.T / n + 1e-3 * torch.eye(n, device=dev)
    symeig([F])
torch.cuda.synchronize()
print(json.dumps({"mode": mode, "done": True, "pid": os.getpid()}), flush=True)
if os.environ.get("EXIT_MAPS"):
    with open("/proc/self/maps") as f, open(os.environ["EXIT_MAPS"], "w") as g:
        g.write(f.read())
if mode == "eig_os":
    sys.stdout.flush()
    sys.stderr.flush()
    os._exit(0)
