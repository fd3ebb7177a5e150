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


def test_gpus_2_mixed_reports_edge_balanced_shards():
    """Config 5's launch: both ranks build the same global batches and shard
    them by edges; the line carries every batch's per-rank edge loads (each
    rank's own count of its first shard is checked against them in-run)."""
    r = _run(["--gpus", "2", "--dry-run", "--graphs", "mixed", "--batches", "2"])
    sh = r["shards"]
    assert r["config"]["global_batch"] == 128
    assert len(sh["rank_edge_loads"]) == 2 and all(len(x) == 2 for x in sh["rank_edge_loads"])
    for loads, sizes in zip(sh["rank_edge_loads"], sh["rank_graphs"]):
        assert sum(sizes) == 128
        assert max(loads) <= 1.1 * sum(loads) / 2
    r = _run(["--gpus", "2", "--dry-run", "--batches", "2"])  # residue graphs: contiguous halves
    assert r["shards"]["balanced"] == [False, False] and r["shards"]["rank_graphs"] == [[64, 64], [64, 64]]
