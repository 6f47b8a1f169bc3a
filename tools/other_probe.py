"""Probe: bench.other_config('lenet') in a fresh process, with more warmup, and after
the MLP's records were allocated and freed (the order bench.py runs it in)."""
import json
import sys

import torch

sys.path.insert(0, ".")
import bench  # noqa: E402

dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
torch.cuda.set_stream(torch.cuda.Stream(dev))
which = sys.argv[1]
if which == "fresh":
    r = bench.other_config("lenet", dev, steps=20, warmup=2)
elif which == "warm":
    r = bench.other_config("lenet", dev, steps=20, warmup=8)
elif which == "twice":
    bench.other_config("lenet", dev, steps=20, warmup=2)
    r = bench.other_config("lenet", dev, steps=20, warmup=2)
print(which, json.dumps({k: r[k] for k in ("value", "ms_per_step")}), r["breakdown"])
