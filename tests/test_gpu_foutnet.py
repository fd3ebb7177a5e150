"""GPU parity of the MI355X FoutNet path (dr_fout_graph_pass + dr_reduce_update,
generic CSR kernels for FoutLayer) against the reference goldens and the CPU
oracle.  Tolerance: 1e-4 (north_star, fp32)."""

from __future__ import annotations

import numpy as np
import pytest
import torch
from _util import assert_grad_close, golden_batch, golden_grads, golden_state_dict

from deeprank2_amd.engine import FusedTrainStep
from deeprank2_amd.fused import BatchHandle
from deeprank2_amd.neuralnets.gnn import foutnet as amd
from deeprank2_amd.store import GraphStore, pack_graphs, records_from_batch
from oracle import data_ref, gnn_ref
from oracle import pyg_ops as P

pytestmark = pytest.mark.gpu
TOL = dict(rtol=1e-4, atol=1e-4)
DEV = "cuda:0"


def _synthetic(n, seed, **kw):
    from deeprank2_amd.utils.synthetic import make_dataset

    return [data_ref.synthetic_to_data(g, f"s{i}") for i, g in enumerate(make_dataset(n, seed=seed, **kw))]


def _pair(f, out, seed):
    torch.manual_seed(seed)
    model_o = gnn_ref.FoutNet(f, out)
    model = amd.FoutNet(f, out)
    model.load_state_dict(model_o.state_dict())
    return model_o, model.to(DEV)


def test_foutnet_module_vs_reference_golden(golden):
    z = golden("foutnet_synth")
    m = amd.FoutNet(30, 1)
    m.load_state_dict(golden_state_dict(z))
    m = m.to(DEV).eval()
    with torch.no_grad():
        out = m(golden_batch(z)).cpu().numpy()
    np.testing.assert_allclose(out, z["out/eval"], **TOL)
    m.train()
    out = m(golden_batch(z))
    loss = torch.nn.functional.mse_loss(out.reshape(-1), torch.from_numpy(z["in/y"]).to(DEV))
    loss.backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), z["out/train"], **TOL)
    assert float(loss.detach()) == pytest.approx(float(z["loss"]), rel=1e-4)
    ref = golden_grads(z)
    for n, p in m.named_parameters():
        assert_grad_close(p.grad.cpu().numpy(), ref[n], err_msg=n)


def test_foutnet_testhdf5_nan_path_vs_golden(golden):
    """test.hdf5: one depth-0 cluster per graph -> the pooled node has no
    out-edge -> mean(empty) = NaN (foutnet.py:58) -> NaN predictions."""
    z = golden("foutnet_testhdf5")
    m = amd.FoutNet(50, 2)
    m.load_state_dict(golden_state_dict(z))
    m = m.to(DEV).eval()
    with torch.no_grad():
        out = m(golden_batch(z)).cpu().numpy()
    ref = z["out/eval"]
    assert np.isnan(ref).any()
    np.testing.assert_array_equal(np.isnan(out), np.isnan(ref))
    np.testing.assert_allclose(out, ref, equal_nan=True, **TOL)


def test_foutnet_nan_gradients_match_oracle(golden):
    """Backward through the NaN path: the same parameters end up NaN."""
    z = golden("foutnet_testhdf5")
    model_o = gnn_ref.FoutNet(50, 2)
    model_o.load_state_dict(golden_state_dict(z))
    m = amd.FoutNet(50, 2)
    m.load_state_dict(golden_state_dict(z))
    m = m.to(DEV)
    model_o(golden_batch(z)).sum().backward()
    m(golden_batch(z)).sum().backward()
    ref = dict(model_o.named_parameters())
    for n, p in m.named_parameters():
        g, r = p.grad.cpu().numpy(), ref[n].grad.numpy()
        np.testing.assert_array_equal(np.isnan(g), np.isnan(r), err_msg=n)
        np.testing.assert_allclose(g, r, equal_nan=True, rtol=1e-4, atol=1e-5, err_msg=n)


@pytest.mark.parametrize("force_layers", [False, True])
def test_foutnet_nan_gradients_match_oracle_both_paths(golden, force_layers):
    """The NaN backward through the graph pass and through the layer-level path
    (layered.py, FoutLayer autograd): a pooled node without out-edges adds
    neither its NaN mean nor its gradient to conv2.wn (foutnet.py:56-58)."""
    from types import SimpleNamespace

    z = golden("foutnet_testhdf5")
    model_o = gnn_ref.FoutNet(50, 2)
    model_o.load_state_dict(golden_state_dict(z))
    m = amd.FoutNet(50, 2)
    m.load_state_dict(golden_state_dict(z))
    m = m.to(DEV)
    bat = golden_batch(z)
    model_o(bat).sum().backward()
    h = BatchHandle(GraphStore(pack_graphs(records_from_batch(golden_batch(z))), DEV), np.arange(4, dtype=np.int32))
    h.force_layers = force_layers
    m(SimpleNamespace(_dr_handle=h)).sum().backward()
    ref = dict(model_o.named_parameters())
    for n, p in m.named_parameters():
        g, r = p.grad.cpu().numpy(), ref[n].grad.numpy()
        np.testing.assert_array_equal(np.isnan(g), np.isnan(r), err_msg=n)
        np.testing.assert_allclose(g, r, equal_nan=True, rtol=1e-4, atol=1e-5, err_msg=n)


def test_foutnet_mixed_lds_layouts_vs_oracle():
    """A batch whose largest graph (N~265) only fits the narrow LDS layout, so
    the launch reserves the narrow size, and graphs (N~235) whose wide layout
    fits 160 KiB but not that launch: every graph must take the layout its
    launch reserved.  Forward + MSE gradients vs the oracle."""
    from deeprank2_amd.utils.synthetic import make_dataset

    gs = make_dataset(1, seed=6, n_lo=262, n_hi=268, mean_degree=15.0) + make_dataset(2, seed=3, n_lo=230, n_hi=238, mean_degree=15.0)
    datas = [data_ref.synthetic_to_data(g, f"m{i}") for i, g in enumerate(gs)]
    h = BatchHandle(GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV), np.arange(3, dtype=np.int32))
    launch = amd.SPEC.lds(*h.max_sizes, 30, int(h.store.packed.transpose_aliased), 1)
    assert launch <= 160 * 1024  # the fused kernel runs, not the layer path
    model_o, model = _pair(30, 1, seed=8)
    bat_o = P.Batch.from_data_list([d.clone() for d in datas])
    out_o = model_o(bat_o)
    torch.nn.functional.mse_loss(out_o.reshape(-1), bat_o.y).backward()
    from types import SimpleNamespace

    out = model(SimpleNamespace(_dr_handle=h))
    torch.nn.functional.mse_loss(out.reshape(-1), bat_o.y.to(DEV)).backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), out_o.detach().numpy(), equal_nan=True, **TOL)
    ref = dict(model_o.named_parameters())
    for n, p in model.named_parameters():
        assert_grad_close(p.grad.cpu().numpy(), ref[n].grad.numpy(), err_msg=n)


def test_foutnet_autograd_vs_oracle_mixed_clusters():
    """Isolated nodes (NaN rows dropped by the depth-0 scatter_max), several
    depth-1 clusters, CE loss over 3 classes."""
    datas = _synthetic(8, seed=21, n_lo=25, n_hi=60, mean_degree=7.0)
    for i, d in enumerate(datas):
        keep = (d.edge_index[0] != 3) & (d.edge_index[1] != 3)  # node 3 isolated everywhere
        d.edge_index = d.edge_index[:, keep]
        d.edge_attr = d.edge_attr[keep]
        if i % 2:
            k = len(d.cluster1)
            d.cluster1 = torch.tensor([j % 2 for j in range(k)], dtype=torch.long) if k > 1 else d.cluster1
        d.y = torch.tensor([float(i % 3)])
    model_o, model = _pair(30, 3, seed=5)
    bat_o = P.Batch.from_data_list([d.clone() for d in datas])
    out_o = model_o(bat_o)
    assert not torch.isnan(out_o).any()
    torch.nn.functional.cross_entropy(out_o, bat_o.y.long()).backward()
    out = model(P.Batch.from_data_list(datas))
    torch.nn.functional.cross_entropy(out, bat_o.y.long().to(DEV)).backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), out_o.detach().numpy(), **TOL)
    ref = dict(model_o.named_parameters())
    for n, p in model.named_parameters():
        assert_grad_close(p.grad.cpu().numpy(), ref[n].grad.numpy(), err_msg=n)


def test_foutlayer_arbitrary_edges_vs_oracle():
    """Layer API on an asymmetric edge list with self loops, duplicates and
    a node without out-edges (NaN row)."""
    gen = torch.Generator().manual_seed(5)
    x = torch.randn(41, 12, generator=gen)
    ei = torch.randint(0, 41, (2, 260), generator=gen)
    ei = ei[:, ei[0] != 7]
    ei = torch.cat([ei, torch.tensor([[3, 3, 3, 9], [3, 3, 4, 9]])], 1)
    torch.manual_seed(2)
    lo = gnn_ref.FoutLayer(12, 16)
    la = amd.FoutLayer(12, 16)
    la.load_state_dict(lo.state_dict())
    la = la.to(DEV)
    xo = x.clone().requires_grad_(True)
    xa = x.to(DEV).requires_grad_(True)
    zo = lo(xo, ei)
    za = la(xa, ei.to(DEV))
    gz = torch.randn(zo.shape, generator=gen)
    (zo.nan_to_num(0.0) * gz).sum().backward()
    (za.nan_to_num(0.0) * gz.to(DEV)).sum().backward()
    assert torch.isnan(zo[7]).all() and torch.isnan(za[7].cpu()).all()
    np.testing.assert_allclose(za.detach().cpu().numpy(), zo.detach().numpy(), equal_nan=True, **TOL)
    np.testing.assert_allclose(xa.grad.cpu().numpy(), xo.grad.numpy(), **TOL)
    for n, p in la.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), dict(lo.named_parameters())[n].grad.numpy(), err_msg=n, **TOL)


def test_foutnet_fused_train_step_vs_oracle():
    """FusedTrainStep (graph pass with in-kernel MSE + reduce/Adam) against the
    oracle forward/backward and torch.optim.Adam."""
    datas = _synthetic(24, seed=3, n_lo=30, n_hi=70, mean_degree=10.0)
    model_o, model = _pair(30, 1, seed=9)
    model.train()
    bat = P.Batch.from_data_list([d.clone() for d in datas])
    out_o = model_o(bat)
    loss_o = torch.nn.functional.mse_loss(out_o.reshape(-1), bat.y)
    loss_o.backward()
    store = GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)
    h = BatchHandle(store, np.arange(24))
    step = FusedTrainStep(model)
    before = [p.detach().clone() for p in step.params]
    loss, out = step.step(h)
    np.testing.assert_allclose(out.cpu().numpy(), out_o.detach().numpy(), **TOL)
    assert float(loss) == pytest.approx(float(loss_o.detach()), rel=1e-4)
    grads = dict(zip(amd.PARAM_NAMES, step.grads))
    for n, p in model_o.named_parameters():
        assert_grad_close(grads[n].cpu().numpy(), p.grad.numpy(), err_msg=n)
    ref = [torch.nn.Parameter(b) for b in before]
    for r, g in zip(ref, step.grads):
        r.grad = g.detach().clone()
    torch.optim.Adam(ref, lr=1e-3, weight_decay=1e-5).step()
    for n, r, p in zip(amd.PARAM_NAMES, ref, step.params):
        np.testing.assert_allclose(p.detach().cpu().numpy(), r.detach().cpu().numpy(), rtol=1e-5, atol=1e-7, err_msg=n)


def test_foutnet_captured_replay_and_determinism():
    datas = _synthetic(32, seed=12)
    store = GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)
    hs = [BatchHandle(store, np.arange(16)), BatchHandle(store, np.arange(16, 32))]
    torch.manual_seed(3)
    m1 = amd.FoutNet(30, 1).to(DEV).train()
    m2 = amd.FoutNet(30, 1).to(DEV).train()
    m2.load_state_dict(m1.state_dict())
    s1, s2 = FusedTrainStep(m1), FusedTrainStep(m2)
    graphs = [s2.capture(h) for h in hs]
    for i in range(6):
        l1, _ = s1.step(hs[i % 2])
        graphs[i % 2].replay()
        torch.cuda.synchronize()
        assert torch.equal(l1, s2.loss_out), i
    for a, b in zip(s1.params, s2.params):
        assert torch.equal(a, b)


def test_foutnet_cpu_model_raises():
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        amd.FoutNet(30, 1)(P.Batch.from_data_list(_synthetic(1, seed=1)))


def test_foutnet_fused_train_step_vs_oracle_config3_batch64():
    """BASELINE configs[2] shape: 64 synthetic residue graphs (N~200, E~3k,
    F=30, Fe=3) through FusedTrainStep — forward, MSE, backward, Adam — for
    three consecutive steps: each step's outputs, loss and gradients against
    the oracle (foutnet.py:48-66,99-118) run on the same weights, and the
    fused Adam against torch.optim.Adam carrying the same state.  Pooled nodes
    without an out-edge would give NaN rows (mean(empty), foutnet.py:58): NaN
    positions must agree, the rest within 1e-4."""
    from deeprank2_amd.utils.synthetic import make_dataset

    datas = [data_ref.synthetic_to_data(g, f"c{i}") for i, g in enumerate(make_dataset(64, seed=0))]
    model_o, model = _pair(30, 1, seed=31)
    model.train()
    store = GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)
    h = BatchHandle(store, np.arange(64))
    step = FusedTrainStep(model)
    by_name = dict(zip(amd.PARAM_NAMES, step.params))
    adam_sd = None
    for it in range(3):
        with torch.no_grad():  # the oracle on the fused step's current weights
            for n, po in model_o.named_parameters():
                po.copy_(by_name[n].detach().cpu())
        model_o.zero_grad()
        bat = P.Batch.from_data_list([d.clone() for d in datas])
        out_o = model_o(bat)
        loss_o = torch.nn.functional.mse_loss(out_o.reshape(-1), bat.y)
        loss_o.backward()
        before = [p.detach().clone() for p in step.params]
        loss, out = step.step(h)
        o, r = out.cpu().numpy(), out_o.detach().numpy()
        np.testing.assert_array_equal(np.isnan(o), np.isnan(r), err_msg=f"step {it}")
        # this seeded batch has no pooled node without out-edges, so every step
        # is finite and checked in full (a NaN batch would end the trajectory
        # and shrink the test to a NaN-position check: fail loudly instead)
        assert np.isfinite(r).all() and np.isfinite(o).all(), f"step {it}: the configs[2] batch must stay finite"
        np.testing.assert_allclose(o, r, **TOL)
        assert float(loss) == pytest.approx(float(loss_o.detach()), rel=1e-4)
        grads = dict(zip(amd.PARAM_NAMES, step.grads))
        for n, p in model_o.named_parameters():
            assert_grad_close(grads[n].cpu().numpy(), p.grad.numpy(), err_msg=f"{n} step {it}")
        ref = [torch.nn.Parameter(b) for b in before]
        ref_opt = torch.optim.Adam(ref, lr=1e-3, weight_decay=1e-5)
        if adam_sd is not None:
            ref_opt.load_state_dict(adam_sd)
        for rr, g in zip(ref, step.grads):
            rr.grad = g.detach().clone()
        ref_opt.step()
        for n, rr, p in zip(amd.PARAM_NAMES, ref, step.params):
            np.testing.assert_allclose(p.detach().cpu().numpy(), rr.detach().cpu().numpy(), rtol=1e-5, atol=1e-7, err_msg=f"{n} step {it}")
        adam_sd = step.adam_state_dict()
