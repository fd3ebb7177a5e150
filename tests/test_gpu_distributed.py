"""Data-parallel FusedTrainStep on the GPU: 2 ranks (child processes, gloo,
sharing cuda:0) against one process on the whole global batch — same losses
and parameters after 3 Adam steps (fp32 reorder tolerance)."""

from __future__ import annotations

import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _launch(model_name, world, out, **extra_env):
    port = _port()
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), OMP_NUM_THREADS="2", **extra_env)
        procs.append(subprocess.Popen([sys.executable, os.path.join(HERE, "ddp_worker.py"), model_name, out], env=env))
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=240))
        except subprocess.TimeoutExpired:
            p.kill()
            rcs.append(-9)
    assert rcs == [0] * world, rcs


@pytest.mark.parametrize("model_name", ["ginet", "foutnet"])
def test_two_ranks_match_single_process(tmp_path, model_name):
    one, two = str(tmp_path / "w1.npz"), str(tmp_path / "w2.npz")
    _launch(model_name, 1, one)
    _launch(model_name, 2, two)
    a, b = np.load(one), np.load(two)
    np.testing.assert_allclose(b["loss"], a["loss"], rtol=1e-5)
    # last step's all-reduced gradients: normwise fp32 reorder tolerance
    np.testing.assert_allclose(b["grad"], a["grad"], rtol=1e-4, atol=1e-6 * float(np.abs(a["grad"]).max()))
    # parameters after 3 Adam steps (lr 1e-3): a near-zero gradient entry may
    # flip sign under reordering, moving that entry by up to ~lr per step
    for k in a.files:
        if k.startswith("p"):
            np.testing.assert_allclose(b[k], a[k], rtol=0, atol=3e-3, err_msg=k)
            assert np.mean(np.abs(b[k] - a[k]) < 1e-6) > 0.95, k


@pytest.mark.parametrize(("model_name", "acc"), [("ginet", "0"), ("vanilla", "0"), ("ginet", "1")])
def test_two_ranks_bit_identical_to_summed_shards(tmp_path, model_name, acc):
    """Two gloo ranks against one process that runs the same two shards one
    after another and sums their gradient buffers (the all-reduce's sum of two
    operands, order-free) before one Adam update: losses, all-reduced gradients
    and parameters after 3 steps agree bit for bit.  VanillaNetwork runs its
    shards of 12 graphs on 4 workgroups per graph (split partial rows).
    acc: GINet's accumulating pass (3 workgroups per shard, one row each)
    under the same all-reduce."""
    emu, two = str(tmp_path / "emu.npz"), str(tmp_path / "w2.npz")
    _launch(model_name, 1, emu, DR_DDP_EMULATE="2", DR_DDP_ACC=acc)
    _launch(model_name, 2, two, DR_DDP_ACC=acc)
    a, b = np.load(emu), np.load(two)
    for k in a.files:
        np.testing.assert_array_equal(b[k], a[k], err_msg=k)


def test_rccl_captured_ddp_step_matches_plain_step(tmp_path):
    """bench.py's N>1 launch path on one GPU: a one-rank RCCL process group,
    every step replayed from a captured HIP graph holding the graph pass, the
    gradient reduce, the RCCL all-reduce and Adam — the same losses and
    parameters as the plain single-process step."""
    one, cap = str(tmp_path / "plain.npz"), str(tmp_path / "rccl.npz")
    _launch("ginet", 1, one)
    _launch("ginet", 1, cap, DR_DDP_PG="nccl", DR_DDP_CAPTURE="1")
    a, b = np.load(one), np.load(cap)
    np.testing.assert_allclose(b["loss"], a["loss"], rtol=1e-6)
    np.testing.assert_allclose(b["grad"], a["grad"], rtol=1e-6, atol=1e-9)
    for k in a.files:
        if k.startswith("p"):
            np.testing.assert_allclose(b[k], a[k], rtol=1e-6, atol=1e-8, err_msg=k)


@pytest.mark.parametrize("model_name", ["ginet", "vanilla"])
def test_two_ranks_mixed_batch_edge_balanced_bit_identical(tmp_path, model_name):
    """Config 5: global batches of residue, SRV-like and
    atom-level graphs sharded over two ranks by edge bin packing.  Losses,
    all-reduced gradients, parameters after 3 steps and the last step's
    predictions gathered back into global-batch order agree bit for bit with
    one process running the same two shards and summing their gradients."""
    emu, two = str(tmp_path / "emu.npz"), str(tmp_path / "w2.npz")
    _launch(model_name, 1, emu, DR_DDP_EMULATE="2", DR_DDP_GRAPHS="mixed")
    _launch(model_name, 2, two, DR_DDP_GRAPHS="mixed")
    a, b = np.load(emu), np.load(two)
    loads = a["loads"]
    assert (loads.max(1) < 1.25 * loads.mean(1)).all()
    for k in a.files:
        np.testing.assert_array_equal(b[k], a[k], err_msg=k)


def test_trainer_ddp_captured_epochs_bit_identical(tmp_path):
    """``Trainer(ngpu=2)`` on a one-rank RCCL group: each training epoch
    replayed from one captured HIP graph (graph pass, gradient reduce, the
    RCCL all-reduce and Adam per step; the epoch's losses all-reduced and its
    predictions gathered once) and each validation's forward passes from
    another (epoch.EvalRunner) give the same losses, exported predictions and
    final parameters, bit for bit, as the per-batch loop."""
    from deeprank2_amd.utils import synthetic as S

    tr, va = str(tmp_path / "train.hdf5"), str(tmp_path / "valid.hdf5")
    S.write_hdf5(tr, S.make_dataset(23, seed=41, n_lo=25, n_hi=60, mean_degree=8.0), prefix="tr")
    S.write_hdf5(va, S.make_dataset(9, seed=42, n_lo=25, n_hi=60, mean_degree=8.0), prefix="va")
    res = {}
    for cap in ("1", "0"):
        out = str(tmp_path / f"cap{cap}.npz")
        env = dict(os.environ, DR_TRAINER_CAPTURE=cap, OMP_NUM_THREADS="2")
        p = subprocess.run([sys.executable, os.path.join(HERE, "trainer_ddp_worker.py"), tr, va, out], env=env, timeout=240, check=False)
        assert p.returncode == 0, p.returncode
        res[cap] = np.load(out)
    a, b = res["1"], res["0"]
    assert bool(a["captured_train"]) and bool(a["captured_eval"])
    assert not bool(b["captured_train"]) and not bool(b["captured_eval"])
    assert set(a.files) - {"captured_train", "captured_eval"} == set(b.files) - {"captured_train", "captured_eval"}
    for k in a.files:
        if not k.startswith("captured"):
            np.testing.assert_array_equal(a[k], b[k], err_msg=k)
