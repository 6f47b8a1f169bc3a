"""CPU: `bench.py --gpus N` launches its own N rank processes (no external torchrun),
each with RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / one shared free
MASTER_PORT, without the parent ever initialising HIP; a failing rank ends the job
with its exit code; fewer visible GPUs than ranks is a clear non-zero exit."""
import json
import os
import subprocess
import sys
import time

import torch

from conftest import ROOT

sys.path.insert(0, ROOT)
import bench  # noqa: E402

CHILD_ENV = r"""
import json, os, sys
keys = ["RANK", "LOCAL_RANK", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR", "MASTER_PORT",
        "HSA_ENABLE_IPC_MODE_LEGACY"]
with open(os.path.join(sys.argv[1], "rank%s.json" % os.environ["RANK"]), "w") as f:
    json.dump({k: os.environ.get(k) for k in keys}, f)
"""

CHILD_FAIL = r"""
import os, sys, time
if os.environ["RANK"] == "1":
    sys.exit(3)
time.sleep(60)
"""


def test_spawn_sets_rank_env_and_parent_stays_off_gpu(tmp_path):
    rc = bench.spawn_ranks(3, [], cmd=[sys.executable, "-c", CHILD_ENV, str(tmp_path)],
                           check_devices=False)
    assert rc == 0
    envs = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(3)]
    ports = {e["MASTER_PORT"] for e in envs}
    assert len(ports) == 1 and ports.pop().isdigit()
    for r, e in enumerate(envs):
        assert e["RANK"] == e["LOCAL_RANK"] == str(r)
        assert e["WORLD_SIZE"] == e["LOCAL_WORLD_SIZE"] == "3"
        assert e["MASTER_ADDR"] == "127.0.0.1"
        assert e["HSA_ENABLE_IPC_MODE_LEGACY"] == "0"
    assert not torch.cuda.is_initialized()


def test_failing_rank_ends_the_job_with_its_code():
    t0 = time.time()
    rc = bench.spawn_ranks(3, [], cmd=[sys.executable, "-c", CHILD_FAIL], check_devices=False)
    assert rc == 3
    assert time.time() - t0 < 40  # the sleeping ranks were terminated, not waited for


def _run_bench(args, env_extra=None):
    env = dict(os.environ, **(env_extra or {}))
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        if env_extra is None or k not in env_extra:
            env.pop(k, None)
    env["HIP_VISIBLE_DEVICES"] = ""
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, env=env,
                          capture_output=True, text=True, timeout=300)


def test_bench_gpus_n_without_enough_gpus_exits_nonzero():
    p = _run_bench(["--gpus", "2"])
    assert p.returncode == 2
    assert "only 0 GPU(s) visible" in p.stderr
    assert p.stdout.strip() == ""  # no bench line from a run that did not happen


def test_bench_world_size_mismatch_exits_nonzero():
    p = _run_bench(["--gpus", "2"], {"WORLD_SIZE": "4", "RANK": "0", "LOCAL_RANK": "0"})
    assert p.returncode == 2
    assert "WORLD_SIZE=4" in p.stderr


def test_workload_shapes():
    # N = 1: C2 (batch 4096, 60,000 images); N > 1: C4's per-rank shard (8,192 rows of a
    # global batch of N x 8,192 = 65,536 at N = 8); C3 LeNet-5 at batch 1024
    assert bench.SHAPES[("mlp", 1)] == (4096, 60000)
    assert bench.SHAPES[("mlp", 2)][0] * 8 == 65536
    assert bench.SHAPES[("lenet", 1)][0] == 1024
    assert bench.flops_per_image(bench.CONFIGS["mlp"]) == 650402
    assert bench.flops_per_image(bench.CONFIGS["lenet"]) == 3110740


def test_strong_scaling_workload():
    # 65,536 x 64 images in global batches of 65,536, split over N ranks
    for n in (1, 2, 4, 8):
        batch, images = bench.workload("mlp", n, strong=True)
        assert batch * n == 65536 and images * n == 65536 * 64
    assert bench.workload("mlp", 1) == bench.SHAPES[("mlp", 1)]
    assert bench.workload("mlp", 4) == bench.SHAPES[("mlp", 2)]


def test_cpu_e2e_baseline_runs():
    v, threads, sample = bench.cpu_e2e_baseline("mlp", 1024, 256, budget_s=0.2, threads=1)
    assert v > 0 and threads == 1 and "Categorical" in sample
