"""The one-launch GINet training step (``dr_ginet_train_step``: graph pass,
then the gradient reduction and Adam by the last workgroups to finish, in
the same launch, opt-in ``FusedTrainStep.fuse_update``) against the two-launch step (``dr_ginet_graph_pass`` +
``dr_reduce_update``).  Both run the same fixed-order arithmetic
(``csrc/reduce_common.h``), so parameters, Adam moments, gradients, loss and
outputs must agree bit for bit — over batch sizes below, at and above the
64 in-launch reducers, with hash dropout, and replayed from a HIP graph.  The
two-launch step itself is checked against the oracle in test_gpu_trainer /
test_gpu_ginet."""

from __future__ import annotations

import numpy as np
import pytest
import torch

from deeprank2_amd.engine import FusedTrainStep
from deeprank2_amd.fused import BatchHandle
from deeprank2_amd.neuralnets.gnn import ginet as amd
from deeprank2_amd.store import GraphStore, pack_graphs
from deeprank2_amd.utils.synthetic import make_dataset

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _records(n, seed):
    from bench import records

    return records(make_dataset(n, seed=seed))


def _pair(loss="mse", out=1):
    torch.manual_seed(3)
    m1 = amd.GINet(30, out, 3).to(DEV).train()
    m2 = amd.GINet(30, out, 3).to(DEV).train()
    m2.load_state_dict(m1.state_dict())
    m2._drop_seed = m1._drop_seed = 12345  # noqa: SLF001
    one = FusedTrainStep(m1, lr=1e-3, weight_decay=1e-5, loss=loss, max_batch=256)
    two = FusedTrainStep(m2, lr=1e-3, weight_decay=1e-5, loss=loss, max_batch=256)
    one.fuse_update, two.fuse_update = True, False
    return one, two


def _assert_same(one, two, what):
    bad = []
    for k, (a, b) in enumerate(zip(one._state_tensors(), two._state_tensors())):  # noqa: SLF001 - params, moments, counter, grads+loss
        if not torch.equal(a, b):
            bad.append((k, a.numel(), int((a != b).sum()), float((a.double() - b.double()).abs().max())))
    assert not bad, f"{what}: (tensor, numel, n_diff, max|diff|) {bad}; sync {one.sync.tolist()}"
    assert not any(one.sync.tolist()), "arrival counters and flags must be left zero"


@pytest.mark.parametrize("sizes", [(64, 64, 64), (7, 1, 130, 64, 200)])
def test_one_launch_step_bit_identical_to_two_launches(sizes):
    store = GraphStore(pack_graphs(_records(256, 31)), DEV)
    one, two = _pair()
    rng = np.random.default_rng(0)
    for i, b in enumerate(sizes):
        h = BatchHandle(store, rng.permutation(256)[:b].astype(np.int32))
        l1, o1 = one.step(h)
        l2, o2 = two.step(h)
        torch.cuda.synchronize()
        assert torch.equal(o1, o2), f"outputs step {i} (B={b})"
        assert torch.equal(l1, l2), f"loss step {i}"
        _assert_same(one, two, f"state after step {i} (B={b})")


def test_one_launch_step_cross_entropy_bit_identical():
    recs = _records(96, 32)
    for i, r in enumerate(recs):
        r.y = float(i % 3)
    store = GraphStore(pack_graphs(recs), DEV)
    one, two = _pair(loss="ce", out=3)
    for s in range(3):
        h = BatchHandle(store, np.arange(s * 32, s * 32 + 32, dtype=np.int32))
        one.step(h)
        two.step(h)
    torch.cuda.synchronize()
    _assert_same(one, two, "CE steps")


def test_one_launch_step_replays_from_hip_graph():
    store = GraphStore(pack_graphs(_records(128, 33)), DEV)
    one, two = _pair()
    hs = [BatchHandle(store, np.arange(k * 64, k * 64 + 64, dtype=np.int32)) for k in range(2)]
    g = one.capture_sweep(hs)
    for _ in range(3):
        g.replay()
        for h in hs:
            two.step(h)
    torch.cuda.synchronize()
    _assert_same(one, two, "captured one-launch steps vs eager two-launch steps")


def _ras_pair():
    one, two = _pair()
    one.fuse_update = False
    one.ras = True
    return one, two


@pytest.mark.parametrize("sizes", [(64, 64, 64, 64), (7, 1, 130, 64, 200)])
def test_reduce_at_start_step_bit_identical_after_flush(sizes):
    """dr_ginet_ras_step: launch t applies step t-1's reduce + Adam to its share
    of the parameter blocks, hands the new parameters to every workgroup
    (grid-wide, in-launch), then runs pass t.  Every step's outputs equal the
    two-launch step's, and after the epoch-end flush the parameters, moments,
    gradients, loss and step counter are bit-identical; the hand-off counters
    and the pending flag are left zero.  Batch sizes vary (the pending update
    sums the previous pass's rows with its loss scale)."""
    store = GraphStore(pack_graphs(_records(256, 34)), DEV)
    one, two = _ras_pair()
    rng = np.random.default_rng(1)
    for i, b in enumerate(sizes):
        h = BatchHandle(store, rng.permutation(256)[:b].astype(np.int32))
        _l1, o1 = one.step(h)
        _l2, o2 = two.step(h)
        torch.cuda.synchronize()
        assert torch.equal(o1, o2), f"outputs step {i} (B={b})"
    one.flush()
    torch.cuda.synchronize()
    _assert_same(one, two, "after the flush")


def test_reduce_at_start_steps_replay_from_hip_graph():
    store = GraphStore(pack_graphs(_records(128, 35)), DEV)
    one, two = _ras_pair()
    hs = [BatchHandle(store, np.arange(k * 64, k * 64 + 64, dtype=np.int32)) for k in range(2)]
    g = one.capture_sweep(hs)
    for _ in range(3):
        g.replay()
        for h in hs:
            two.step(h)
    one.flush()
    torch.cuda.synchronize()
    _assert_same(one, two, "captured reduce-at-start steps + flush vs eager two-launch steps")


def test_reduce_at_start_pending_update_flushed_before_other_paths():
    """A batch the reduce-at-start launch cannot take (B > 256: the regular
    two-launch step) applies the pending update first, and reading the
    optimizer state flushes it too: the state stays bit-identical to the
    two-launch steps (without the flush the regular step's reduce
    overwrote the pending partials, and the next RAS launch re-applied them)."""
    store = GraphStore(pack_graphs(_records(320, 36)), DEV)
    one, two = _ras_pair()
    rng = np.random.default_rng(2)
    for i, b in enumerate((64, 300, 64, 257, 32)):
        h = BatchHandle(store, rng.permutation(320)[:b].astype(np.int32))
        _l1, o1 = one.step(h)
        _l2, o2 = two.step(h)
        torch.cuda.synchronize()
        assert torch.equal(o1, o2), f"outputs step {i} (B={b})"
    sd1, sd2 = one.adam_state_dict(), two.adam_state_dict()  # flushes the pending update
    for k in sd2["state"]:
        for name in ("exp_avg", "exp_avg_sq"):
            assert torch.equal(sd1["state"][k][name], sd2["state"][k][name]), (k, name)
    _assert_same(one, two, "after B > 256 steps and the optimizer-state flush")


def _piped_pair():
    one, two = _pair()
    one.fuse_update = False
    one.piped = True
    return one, two


@pytest.mark.parametrize("sizes", [(64, 64, 64, 64, 64), (7, 1, 130, 64, 200, 33)])
def test_piped_step_bit_identical_after_flush(sizes):
    """dr_ginet_piped_step: launch t runs step t-1's reduce + Adam on its own
    reducer workgroups beside pass t, whose waves wait for that update only
    right before reading a weight; partials double-buffered.  Every step's
    outputs equal the two-launch step's and after the flush the parameters,
    moments, gradients, loss and step counter are bit-identical; a batch the
    pipelined launch cannot take (B = 200: reducers + graph workgroups over
    224) runs the regular step after flushing the pending update."""
    store = GraphStore(pack_graphs(_records(256, 37)), DEV)
    one, two = _piped_pair()
    rng = np.random.default_rng(3)
    for i, b in enumerate(sizes):
        h = BatchHandle(store, rng.permutation(256)[:b].astype(np.int32))
        _l1, o1 = one.step(h)
        _l2, o2 = two.step(h)
        torch.cuda.synchronize()
        assert torch.equal(o1, o2), f"outputs step {i} (B={b})"
    one.flush()
    torch.cuda.synchronize()
    _assert_same(one, two, "pipelined steps after the flush")


def test_piped_steps_replay_from_hip_graph():
    """Captured sweeps of pipelined steps replayed back to back (the update of
    each sweep's last pass runs in the next replay's first launch), flushed at
    the end: bit-identical to eager two-launch steps."""
    store = GraphStore(pack_graphs(_records(192, 38)), DEV)
    one, two = _piped_pair()
    hs = [BatchHandle(store, np.arange(k * 64, k * 64 + 64, dtype=np.int32)) for k in range(3)]
    g = one.capture_sweep(hs)
    for _ in range(3):
        g.replay()
        for h in hs:
            two.step(h)
    one.flush()
    torch.cuda.synchronize()
    _assert_same(one, two, "captured pipelined steps + flush vs eager two-launch steps")
