"""The accumulating GINet pass (``dr_ginet_acc_pass``, r05): for batches past
the CU count each workgroup runs every R-th graph and sums their gradients on
chip, writing one partial row per workgroup, and ``dr_reduce_update`` sums R
rows instead of B per-graph partials.  Against the per-graph step
(``dr_ginet_graph_pass`` + the reduce, itself checked against the oracle in
test_gpu_trainer / test_gpu_ginet):

* the forward outputs are bit-identical (the same per-graph arithmetic);
* the loss and the gradients are the same sums in another fp32 association:
  loss within 1e-6 relative, every gradient element within 1e-5 of its
  parameter's largest gradient magnitude (fp32, sums of <= 1000 terms);
* with hash dropout, MSE and cross-entropy, ragged graph sizes, one or
  several graphs per workgroup, and replayed from a HIP graph (captured
  replays bit-identical to eager accumulating steps: deterministic).
"""

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
GRAD_TOL = 1e-5  # x max |grad| of the parameter
LOSS_TOL = 1e-6  # relative


def _records(n, seed, classes=0, n_feat=30):
    from bench import records

    # (F > 32: graphs of <= 150 nodes, so the carve with 64-wide Z rows plus
    # the LDS fc1.weight block fits one workgroup)
    kw = {"n_lo": 110, "n_hi": 150} if n_feat > 32 else {}
    recs = records(make_dataset(n, seed=seed, n_feat=n_feat, **kw))
    if classes:
        for i, r in enumerate(recs):
            r.y = float(i % classes)
    return recs


def _pair(loss="mse", out=1, groups=None, f=30):
    torch.manual_seed(5)
    m1 = amd.GINet(f, out, 3).to(DEV).train()
    m2 = amd.GINet(f, out, 3).to(DEV).train()
    m2.load_state_dict(m1.state_dict())
    m2._drop_seed = m1._drop_seed = 777  # noqa: SLF001
    acc = FusedTrainStep(m1, loss=loss, max_batch=64)
    per = FusedTrainStep(m2, loss=loss, max_batch=64)
    acc.acc, acc.acc_groups = True, groups
    per.acc = False
    return acc, per


def _assert_close_grads(acc, per, what):
    for name, ga, gp in zip(amd.PARAM_NAMES, acc.grads, per.grads):
        scale = float(gp.abs().max())
        if scale == 0.0:
            assert torch.equal(ga, gp), f"{what}: {name} (exact zeros)"
            continue
        err = float((ga.double() - gp.double()).abs().max())
        assert err <= GRAD_TOL * scale, f"{what}: {name} max|diff| {err:.3g} vs max|grad| {scale:.3g}"


@pytest.mark.parametrize(("n", "groups", "f"), [(300, None, 30), (1000, None, 30), (64, 7, 30), (40, 1, 30), (300, None, 40)])
def test_acc_pass_matches_per_graph_partials(n, groups, f):
    """(F = 40: the F > 32 kernel, fc1.weight's sums in LDS instead of registers.)"""
    store = GraphStore(pack_graphs(_records(max(n, 64), 41, n_feat=f)), DEV)
    acc, per = _pair(groups=groups, f=f)
    rng = np.random.default_rng(4)
    h = BatchHandle(store, rng.permutation(max(n, 64))[:n].astype(np.int32))
    assert acc._acc_rows(h) > 0 and per._acc_rows(h) == 0  # noqa: SLF001
    la, oa = acc.step(h)
    lp, op = per.step(h)
    torch.cuda.synchronize()
    assert torch.equal(oa, op), "forward outputs"
    assert abs(float(la) - float(lp)) <= LOSS_TOL * abs(float(lp)), (float(la), float(lp))
    _assert_close_grads(acc, per, f"B={n} groups={groups}")


@pytest.mark.parametrize(("n", "f"), [(300, 30), (1000, 30)])
def test_acc_prefetch_layout_bit_identical(n, f):
    """The prefetch layout (weights kept in LDS across a workgroup's graphs,
    graph k+1's inputs DMA'd under graph k's tail) moves data, not
    arithmetic: bit-identical to the accumulating pass without it."""
    store = GraphStore(pack_graphs(_records(n, 44, n_feat=f)), DEV)
    one, _ = _pair(f=f)
    two, _ = _pair(f=f)
    one.acc_prefetch, two.acc_prefetch = True, False
    h = BatchHandle(store, np.arange(n, dtype=np.int32))
    assert one.acc_lds(h) != two.acc_lds(h), "the prefetch layout must be the one taken"
    for _ in range(2):
        l1, o1 = one.step(h)
        l2, o2 = two.step(h)
        torch.cuda.synchronize()
        assert torch.equal(o1, o2) and torch.equal(l1, l2)
    for k, (a, b) in enumerate(zip(one._state_tensors(), two._state_tensors())):  # noqa: SLF001
        assert torch.equal(a, b), f"state tensor {k}"


def test_acc_pass_cross_entropy_ragged_several_steps():
    """CE with 3 classes over batches of varying size (one of them below the
    CU count: auto mode takes the per-graph partials there), 3 steps; the
    parameters stay within Adam-amplified fp32 noise of the per-graph step."""
    store = GraphStore(pack_graphs(_records(600, 42, classes=3)), DEV)
    acc, per = _pair(loss="ce", out=3)
    acc.acc = None  # auto
    rng = np.random.default_rng(5)
    for i, b in enumerate((600, 100, 513)):
        h = BatchHandle(store, rng.permutation(600)[:b].astype(np.int32))
        la, oa = acc.step(h)
        lp, op = per.step(h)
        torch.cuda.synchronize()
        if i == 0:  # same parameters: outputs equal, gradients close
            assert torch.equal(oa, op)
            _assert_close_grads(acc, per, "CE step 0")
        assert abs(float(la) - float(lp)) <= 1e-4 * abs(float(lp)), (i, float(la), float(lp))
    for a, p in zip(acc.params, per.params):
        assert float((a - p).abs().max()) <= 1e-5, "parameters after 3 steps (lr 1e-3)"


def test_acc_steps_replay_from_hip_graph_deterministic():
    """A captured sweep of accumulating steps replayed 3 times equals the same
    steps run eagerly, bit for bit (fixed graph -> workgroup map and order)."""
    store = GraphStore(pack_graphs(_records(1024, 43)), DEV)
    one, _ = _pair()
    two, _ = _pair()
    two.acc = True
    hs = [BatchHandle(store, np.arange(k * 512, k * 512 + 512, dtype=np.int32)) for k in range(2)]
    g = one.capture_sweep(hs)
    for _ in range(3):
        g.replay()
        for h in hs:
            two.step(h)
    torch.cuda.synchronize()
    for k, (a, b) in enumerate(zip(one._state_tensors(), two._state_tensors())):  # noqa: SLF001
        assert torch.equal(a, b), f"state tensor {k}"
