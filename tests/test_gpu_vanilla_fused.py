"""GPU parity of the per-graph fused VanillaNetwork kernel (dr_vanilla_fused_pass,
vanilla_graph.hip) against the CPU oracle (oracle/gnn_ref.py, the op-for-op
restatement of deeprank2/neuralnets/gnn/vanilla_gnn.py) and against the
batch-wide pipeline (dr_vanilla_graph_pass).  Tolerance: 1e-4 (north_star, fp32)."""

from __future__ import annotations

import numpy as np
import pytest
import torch
from _util import assert_grad_close

from deeprank2_amd.engine import FusedTrainStep
from deeprank2_amd.fused import BatchHandle
from deeprank2_amd.neuralnets.gnn import vanilla_gnn as amd
from deeprank2_amd.store import GraphRecord, GraphStore, pack_graphs, records_from_batch
from deeprank2_amd.utils.synthetic import make_dataset
from oracle import data_ref, gnn_ref
from oracle import pyg_ops as P

pytestmark = pytest.mark.gpu
TOL = dict(rtol=1e-4, atol=1e-4)
DEV = "cuda:0"


def _datas(n, seed, fe=3, **kw):
    out = []
    for i, g in enumerate(make_dataset(n, seed=seed, **kw)):
        d = data_ref.synthetic_to_data(g, f"v{i}")
        ea = d.edge_attr[:, :fe]
        if fe > ea.shape[1]:  # extra synthetic edge features (the generator makes 3)
            extra = torch.from_numpy(np.random.default_rng(seed + i).standard_normal((ea.shape[0], fe - ea.shape[1])).astype(np.float32))
            ea = torch.cat([ea, extra], 1)
        d.edge_attr = ea.contiguous()
        d.cluster0 = d.cluster1 = None
        out.append(d)
    return out


def _oracle_step(datas, f, out_dim, fe, seed, loss="mse", y=None):
    torch.manual_seed(seed)
    mo = gnn_ref.VanillaNetwork(f, out_dim, fe)
    bat = P.Batch.from_data_list([d.clone() for d in datas])
    out_o = mo(bat)
    if loss == "mse":
        lo = torch.nn.functional.mse_loss(out_o.reshape(-1), bat.y)
    else:
        lo = torch.nn.functional.cross_entropy(out_o, y)
    lo.backward()
    return mo, out_o.detach(), lo.detach()


def _check(mo, out, out_o, grads):
    np.testing.assert_allclose(out.detach().cpu().numpy(), out_o.numpy(), **TOL)
    for n, p in mo.named_parameters():
        assert_grad_close(grads[n].cpu().numpy(), p.grad.numpy(), err_msg=n)


def _store(datas):
    return GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas)), require_clusters=False), DEV)


@pytest.mark.parametrize("fe", [1, 3, 4])
def test_fused_residue_graphs_train_step_vs_oracle(fe):
    """Batch of 8: the default split runs 4 workgroups per graph."""
    datas = _datas(8, seed=51 + fe, fe=fe)  # ~200 nodes, ~3k directed edges
    mo, out_o, loss_o = _oracle_step(datas, 30, 1, fe, seed=21)
    m = amd.VanillaNetwork(30, 1, fe)
    m.load_state_dict(mo.state_dict())
    step = FusedTrainStep(m.to(DEV).train())
    h = BatchHandle(_store(datas), np.arange(8))
    assert amd.fused_fits(h, 30, fe)
    loss, out = step.step(h)
    assert float(loss) == pytest.approx(float(loss_o), rel=1e-4)
    _check(mo, out, out_o, dict(zip(amd.PARAM_NAMES, step.grads)))


def test_fused_matches_pipeline_and_is_deterministic():
    datas = _datas(12, seed=61, n_lo=40, n_hi=220)
    store = _store(datas)
    torch.manual_seed(5)
    m1 = amd.VanillaNetwork(30, 1, 3).to(DEV)
    m2 = amd.VanillaNetwork(30, 1, 3).to(DEV)
    m2.load_state_dict(m1.state_dict())
    h1, h2 = BatchHandle(store, np.arange(12)), BatchHandle(store, np.arange(12))
    h2.vanilla_pipeline = True
    s1, s2 = FusedTrainStep(m1), FusedTrainStep(m2)
    l1, o1 = s1.step(h1)
    g1 = [g.clone() for g in s1.grads]
    l2, o2 = s2.step(h2)
    np.testing.assert_allclose(o1.cpu().numpy(), o2.cpu().numpy(), **TOL)
    for n, a, b in zip(amd.PARAM_NAMES, g1, s2.grads):
        assert_grad_close(a.cpu().numpy(), b.cpu().numpy(), err_msg=n)
    # bitwise repeatable: fixed-order sums only (no float atomics)
    torch.manual_seed(5)
    m4 = amd.VanillaNetwork(30, 1, 3).to(DEV)
    s4 = FusedTrainStep(m4)
    s4.step(BatchHandle(store, np.arange(12)))
    for a, b in zip(g1, s4.grads):
        assert torch.equal(a, b)


def test_fused_irregular_graphs_classification_vs_oracle():
    """Directed (non-symmetric) edges, self loops, duplicate edges, an isolated
    node, a node with no out-edges, a high-degree hub (> 16 edges per row: several
    chunks) and a single-node graph; CE loss over 3 classes."""
    rng = np.random.default_rng(9)
    recs = []
    for gi, n in enumerate([57, 1, 120, 33]):
        e = max(0, n * 6)
        src = rng.integers(0, n, e)
        dst = rng.integers(0, n, e)
        if n > 10:
            src[:40] = 3  # hub: 40+ out-edges of node 3
            keep = (src != 5) & (dst != 5)  # isolated node 5
            src, dst = src[keep], dst[keep]
            src = np.concatenate([src, [7, 7, 7]])
            dst = np.concatenate([dst, [7, 7, 8]])  # self loops + duplicate
            keep = src != 9  # node 9: no out-edges
            src, dst = src[keep], dst[keep]
        ei = np.stack([src, dst]).astype(np.int64)
        recs.append(GraphRecord(x=rng.standard_normal((n, 30)).astype(np.float32), edge_index=ei, edge_attr=rng.standard_normal((ei.shape[1], 2)).astype(np.float32), y=float(gi % 3), name=f"irr{gi}"))
    store = GraphStore(pack_graphs(recs, require_clusters=False), DEV)
    datas = []
    for r in recs:
        d = P.Data(x=torch.from_numpy(r.x), edge_index=torch.from_numpy(r.edge_index), edge_attr=torch.from_numpy(r.edge_attr), y=torch.tensor([r.y]))
        datas.append(d)
    y = torch.tensor([0, 1, 2, 0])
    mo, out_o, _ = _oracle_step(datas, 30, 3, 2, seed=33, loss="ce", y=y)
    m = amd.VanillaNetwork(30, 3, 2)
    m.load_state_dict(mo.state_dict())
    step = FusedTrainStep(m.to(DEV).train(), loss="ce")
    h = BatchHandle(store, np.arange(4))
    assert amd.fused_fits(h, 30, 2)
    _loss, out = step.step(h)
    _check(mo, out, out_o, dict(zip(amd.PARAM_NAMES, step.grads)))


def test_fused_eval_forward_only_and_capture():
    datas = _datas(16, seed=71)
    store = _store(datas)
    torch.manual_seed(8)
    m = amd.VanillaNetwork(30, 1, 3).to(DEV)
    mo = gnn_ref.VanillaNetwork(30, 1, 3)
    mo.load_state_dict({k: v.cpu() for k, v in m.state_dict().items()})
    with torch.no_grad():
        out = m.eval()(P.Batch.from_data_list(datas))
        out_o = mo.eval()(P.Batch.from_data_list([d.clone() for d in datas]))
    np.testing.assert_allclose(out.cpu().numpy(), out_o.numpy(), **TOL)
    hs = [BatchHandle(store, np.arange(8)), BatchHandle(store, np.arange(8, 16))]
    m2 = amd.VanillaNetwork(30, 1, 3).to(DEV)
    m2.load_state_dict(m.state_dict())
    s1, s2 = FusedTrainStep(m.train()), FusedTrainStep(m2.train())
    graphs = [s2.capture(h) for h in hs]
    for i in range(3):
        l1, _ = s1.step(hs[i % 2])
        graphs[i % 2].replay()
        torch.cuda.synchronize()
        assert torch.equal(l1, s2.loss_out), i
    for a, b in zip(s1.params, s2.params):
        assert torch.equal(a, b)


def _split_step(datas, store, fe, split, state, loss="mse", out_dim=1):
    m = amd.VanillaNetwork(30, out_dim, fe)
    m.load_state_dict(state)
    m = m.to(DEV)
    step = FusedTrainStep(m.train(), loss=loss)
    h = BatchHandle(store, np.arange(len(datas)))
    h.vanilla_split = split
    assert amd.split_k(h, 30, fe) == split
    loss_v, out = step.step(h)
    torch.cuda.synchronize()
    _buf, _offs, sync, _wpack = h.vanilla_fused_scratch()
    assert h.vanilla_sync_ok(), "a hand-off wait gave up"
    assert int(sync.abs().sum()) == 0, "arrival counters not left zero"
    return m, step, loss_v.clone(), out.clone(), [g.clone() for g in step.grads], [p.detach().clone() for p in step.params]


@pytest.mark.parametrize("split", [1, 2, 3, 4])
def test_split_workgroups_per_graph_vs_oracle(split):
    """k workgroups per graph (edge-balanced row ranges, B2 / column sums / dS2 /
    dS1 exchanged in-launch, k partial slab rows per graph) against the oracle:
    forward, loss, every gradient and the Adam step's parameters."""
    datas = _datas(8, seed=83)
    mo, out_o, loss_o = _oracle_step(datas, 30, 1, 3, seed=29)
    _m, step, loss, out, grads, _ = _split_step(datas, _store(datas), 3, split, mo.state_dict())
    assert float(loss) == pytest.approx(float(loss_o), rel=1e-4)
    _check(mo, out, out_o, dict(zip(amd.PARAM_NAMES, grads)))


def test_split_irregular_graphs_and_determinism():
    """Graphs smaller than the split (a single node, 3 nodes: siblings owning
    no rows), a hub row, isolated nodes; CE loss.  Every split agrees with the
    oracle, and a split run repeats bit for bit."""
    rng = np.random.default_rng(19)
    recs = []
    for gi, n in enumerate([1, 3, 150, 64, 2, 200]):
        e = n * 7 if n > 3 else n
        src, dst = rng.integers(0, n, e), rng.integers(0, n, e)
        if n > 60:
            src[:50] = 2  # hub row
            keep = (src != 4) & (dst != 4)
            src, dst = src[keep], dst[keep]
        ei = np.stack([src, dst]).astype(np.int64)
        recs.append(GraphRecord(x=rng.standard_normal((n, 30)).astype(np.float32), edge_index=ei, edge_attr=rng.standard_normal((ei.shape[1], 3)).astype(np.float32), y=float(gi % 2), name=f"s{gi}"))
    store = GraphStore(pack_graphs(recs, require_clusters=False), DEV)
    datas = [P.Data(x=torch.from_numpy(r.x), edge_index=torch.from_numpy(r.edge_index), edge_attr=torch.from_numpy(r.edge_attr), y=torch.tensor([r.y])) for r in recs]
    y = torch.tensor([int(r.y) for r in recs])
    mo, out_o, _ = _oracle_step(datas, 30, 2, 3, seed=41, loss="ce", y=y)
    runs = {}
    for split in (1, 4, 4, 3):
        _m, _step, _l, out, grads, params = _split_step(datas, store, 3, split, mo.state_dict(), loss="ce", out_dim=2)
        _check(mo, out, out_o, dict(zip(amd.PARAM_NAMES, grads)))
        if split in runs:  # bitwise repeatable
            for a, b in zip(runs[split], grads + params):
                assert torch.equal(a, b)
        runs[split] = grads + params


def test_handoff_timeout_is_loud_and_not_sticky():
    """A hand-off wait that gives up (forced here: dr_pass.spin_limit = 1 poll)
    withholds the step: NaN loss, parameters / moments / step counter unchanged,
    the arrival counters still left zero; the next launch clears the per-launch
    flag and trains normally; check_faults() raises once for the epoch."""
    datas = _datas(64, seed=91)  # 64 graphs: 4 workgroups per graph
    store = _store(datas)
    torch.manual_seed(3)
    m = amd.VanillaNetwork(30, 1, 3).to(DEV)
    step = FusedTrainStep(m.train())
    h = BatchHandle(store, np.arange(64))
    h.vanilla_split = 4
    before = [p.detach().clone() for p in step.params]
    step._pass.spin_limit = step._pass_nodrop.spin_limit = 1  # noqa: SLF001
    loss, _ = step.step(h)
    torch.cuda.synchronize()
    # fault[0] was read by the update and cleared by its last block (the next
    # pass reads the packed weights as they are and makes no pack launch)
    assert int(step.fault[0]) == 0 and int(step.fault[1]) >= 1 and int(step.ticket[0]) == 0
    assert torch.isnan(loss).all()
    assert all(torch.isnan(g).all() for g in step.grads)
    for a, b in zip(before, step.params):
        assert torch.equal(a, b)
    assert all(int(t.abs().sum()) == 0 for st in step.states for t in st)
    assert int(step.counter[0]) == 0
    _buf, _offs, sync, _wpack = h.vanilla_fused_scratch()
    assert int(sync[:-1].abs().sum()) == 0, "arrival counters not left zero"
    step._pass.spin_limit = step._pass_nodrop.spin_limit = 0  # noqa: SLF001
    loss2, _ = step.step(h)
    torch.cuda.synchronize()
    assert int(step.fault[0]) == 0 and bool(torch.isfinite(loss2).all())
    assert int(step.counter[0]) == 1
    assert not all(torch.equal(a, b) for a, b in zip(before, step.params))
    with pytest.raises(RuntimeError, match="gave up"):
        step.check_faults()
    step.check_faults()  # the count was reset: no error


def test_packed_weights_kept_current_by_adam():
    """FusedTrainStep keeps one packed weight copy that Adam rewrites as it
    updates the parameters (dr_adam.mirror), so the pass makes no pack launch
    (DR_PASS_WPACK_CURRENT): steps bitwise equal to packing every launch, the
    copy equal to a fresh pack, and parameters loaded between steps repacked
    (torch version counters)."""
    from deeprank2_amd import _lib

    datas = _datas(16, seed=95)
    store = _store(datas)
    torch.manual_seed(4)
    m1 = amd.VanillaNetwork(30, 1, 3).to(DEV)
    m2 = amd.VanillaNetwork(30, 1, 3).to(DEV)
    m2.load_state_dict(m1.state_dict())
    s1, s2 = FusedTrainStep(m1.train()), FusedTrainStep(m2.train())
    s2.packed_mirror = False
    h1, h2 = BatchHandle(store, np.arange(16)), BatchHandle(store, np.arange(16))
    assert amd.split_k(h1, 30, 3) > 1

    def same():
        for i in range(3):
            l1, o1 = s1.step(h1)
            l2, o2 = s2.step(h2)
            assert torch.equal(l1, l2) and torch.equal(o1, o2), i
        for a, b in zip(s1.params, s2.params):
            assert torch.equal(a, b)
        fresh = torch.empty_like(s1.wpack[0])
        _lib.check(_lib.load().dr_vanilla_wpack(s1._w, 30, 3, fresh.data_ptr(), _lib.stream_ptr(DEV)), "dr_vanilla_wpack")  # noqa: SLF001
        assert torch.equal(fresh, s1.wpack[0])

    same()
    assert s2.wpack is None
    torch.manual_seed(7)
    state = amd.VanillaNetwork(30, 1, 3).state_dict()
    m1.load_state_dict(state)
    m2.load_state_dict(state)
    same()
    torch.cuda.synchronize()
    assert int(s1.ticket[0]) == 0 and int(s1.fault[0]) == 0
