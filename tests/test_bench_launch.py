"""bench.py's multi-GPU launch path, without a GPU.

``python bench.py --gpus N`` outside torch.distributed.run must start N rank
processes (as a child ``torch.distributed.run``) before anything touches the
GPU, and rank 0's line must report the world the ranks actually formed.
``--dry-run`` stops each rank after joining a gloo group, so the launcher
itself is exercised here; the GPU leg is tests/test_gpu_bench.py."""

from __future__ import annotations

import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env_extra=None):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT")}
    env.update(env_extra or {})
    out = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True, env=env, timeout=240, check=True)
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out.stdout + out.stderr
    return json.loads(lines[0])


def test_gpus_2_launches_two_ranks():
    r = _run(["--gpus", "2", "--dry-run"])
    assert r["n_gpus"] == 2 and r["world_size"] == 2
    assert r["backend"] == "gloo"
    assert r["config"]["parallelism"] == "dp2"
    assert r["metric"].startswith("graphs/sec")


def test_gpus_1_is_one_process():
    r = _run(["--dry-run"])
    assert r["n_gpus"] == 1 and r["config"]["parallelism"] == "dp1"
