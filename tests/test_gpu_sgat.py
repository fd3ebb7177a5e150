"""GPU parity of the MI355X SGAT path (dr_sgat_graph_pass + dr_reduce_update;
dr_spmm_csr_w + linear kernels for SGraphAttentionLayer) against goldens
generated from the reference's sgat.py and the CPU oracle.  Tolerance: 1e-4
(north_star, fp32)."""

from __future__ import annotations

import numpy as np
import pytest
import torch
from _util import assert_grad_close, golden_batch, golden_grads, golden_state_dict

from deeprank2_amd.engine import FusedTrainStep
from deeprank2_amd.fused import BatchHandle
from deeprank2_amd.neuralnets.gnn import sgat as amd
from deeprank2_amd.store import GraphStore, pack_graphs, records_from_batch
from oracle import data_ref, gnn_ref
from oracle import pyg_ops as P

pytestmark = pytest.mark.gpu
TOL = dict(rtol=1e-4, atol=1e-4)
DEV = "cuda:0"


def _synthetic(n, seed, **kw):
    from deeprank2_amd.utils.synthetic import make_dataset

    out = [data_ref.synthetic_to_data(g, f"s{i}") for i, g in enumerate(make_dataset(n, seed=seed, **kw))]
    for d in out:
        d.edge_attr = d.edge_attr[:, :1].contiguous()
    return out


def _loss(out, y, kind):
    return torch.nn.functional.mse_loss(out.reshape(-1), y) if kind == "mse" else torch.nn.functional.cross_entropy(out, y.long())


@pytest.mark.parametrize("name,f,out_dim", [("sgat_1atn", 50, 1), ("sgat_synth", 30, 2)])
def test_sgat_module_vs_reference_golden(golden, name, f, out_dim):
    z = golden(name)
    kind = str(z["meta/loss"])
    m = amd.SGAT(f, out_dim)
    m.load_state_dict(golden_state_dict(z))
    m = m.to(DEV).eval()
    with torch.no_grad():
        out = m(golden_batch(z)).cpu().numpy()
    np.testing.assert_allclose(out, z["out/eval"], **TOL)
    m.train()
    out = m(golden_batch(z))
    loss = _loss(out, torch.from_numpy(z["in/y"]).to(DEV), kind)
    loss.backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), z["out/train"], **TOL)
    assert float(loss.detach()) == pytest.approx(float(z["loss"]), rel=1e-4)
    ref = golden_grads(z)
    for n, p in m.named_parameters():
        assert_grad_close(p.grad.cpu().numpy(), ref[n], err_msg=n)


@pytest.mark.parametrize("name", ["sgat_layer", "sgat_layer_directed"])
def test_sgat_layer_vs_reference_golden(golden, name):
    z = golden(name)
    la = amd.SGraphAttentionLayer(12, 16, undirected=bool(z["meta/undirected"]))
    la.load_state_dict({k[6:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("param/")})
    la = la.to(DEV)
    x = torch.from_numpy(z["in/x"]).to(DEV).requires_grad_(True)
    out = la(x, torch.from_numpy(z["in/edge_index"]).to(DEV), torch.from_numpy(z["in/edge_attr"]).to(DEV))
    (out * torch.from_numpy(z["in/gz"]).to(DEV)).sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), z["out/z"], **TOL)
    np.testing.assert_allclose(x.grad.cpu().numpy(), z["grad/x"], **TOL)
    for n, p in la.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), z["grad/" + n], err_msg=n, **TOL)


def test_sgat_autograd_vs_oracle_mixed_clusters():
    """Isolated nodes (bias-only rows), several depth-1 clusters, CE over 3 classes."""
    datas = _synthetic(8, seed=23, n_lo=25, n_hi=60, mean_degree=7.0)
    for i, d in enumerate(datas):
        keep = (d.edge_index[0] != 3) & (d.edge_index[1] != 3)
        d.edge_index = d.edge_index[:, keep]
        d.edge_attr = d.edge_attr[keep]
        if i % 2:
            k = len(d.cluster1)
            d.cluster1 = torch.tensor([j % 2 for j in range(k)], dtype=torch.long) if k > 1 else d.cluster1
        d.y = torch.tensor([float(i % 3)])
    torch.manual_seed(5)
    model_o = gnn_ref.SGAT(30, 3)
    model = amd.SGAT(30, 3)
    model.load_state_dict(model_o.state_dict())
    model = model.to(DEV)
    bat_o = P.Batch.from_data_list([d.clone() for d in datas])
    out_o = model_o(bat_o)
    torch.nn.functional.cross_entropy(out_o, bat_o.y.long()).backward()
    out = model(P.Batch.from_data_list(datas))
    torch.nn.functional.cross_entropy(out, bat_o.y.long().to(DEV)).backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), out_o.detach().numpy(), **TOL)
    ref = dict(model_o.named_parameters())
    for n, p in model.named_parameters():
        assert_grad_close(p.grad.cpu().numpy(), ref[n].grad.numpy(), err_msg=n)


def test_sgat_fused_train_step_vs_oracle():
    datas = _synthetic(24, seed=4, n_lo=30, n_hi=70, mean_degree=10.0)
    torch.manual_seed(9)
    model_o = gnn_ref.SGAT(30, 1)
    model = amd.SGAT(30, 1)
    model.load_state_dict(model_o.state_dict())
    model = model.to(DEV).train()
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


def test_sgat_needs_one_edge_feature():
    datas = _synthetic(2, seed=1)
    for d in datas:
        d.edge_attr = torch.cat([d.edge_attr, d.edge_attr], 1)
    m = amd.SGAT(30, 1).to(DEV)
    with pytest.raises(ValueError, match="one edge feature"):
        m(P.Batch.from_data_list(datas))
    la = amd.SGraphAttentionLayer(30, 16).to(DEV)
    with pytest.raises(ValueError, match="one edge feature"):
        la(datas[0].x.to(DEV), datas[0].edge_index.to(DEV), datas[0].edge_attr.to(DEV))


def test_sgat_adam_trajectory_vs_oracle_replay():
    """40 Adam steps of the fused SGAT step over 4 resident mini-batches of
    residue graphs (edge weight = the distance feature, as in the bench)
    against the oracle (sgat.py:56-133) trained by torch.optim.Adam on the
    same batches from the same initialisation: the per-step losses and the
    final parameters agree.  The reference itself starts from a very large
    loss (~3e4 on the bench's batches: distance-weighted neighbour means) and
    is still at ~30-150 after a few hundred steps (an oracle replay of the
    bench's first 230 steps: 33461 -> 36.1), so the bench's SGAT final loss of
    ~140 is this trajectory, not a divergence of the kernels."""
    from deeprank2_amd.utils.synthetic import make_dataset

    gs = make_dataset(64, seed=77)
    datas = [data_ref.synthetic_to_data(g, f"t{i}") for i, g in enumerate(gs)]
    for d in datas:
        d.edge_attr = d.edge_attr[:, :1].contiguous()
    batches = [list(range(k * 16, (k + 1) * 16)) for k in range(4)]
    torch.manual_seed(12)
    model_o = gnn_ref.SGAT(30, 1)
    model = amd.SGAT(30, 1)
    model.load_state_dict(model_o.state_dict())
    model = model.to(DEV).train()
    opt_o = torch.optim.Adam(model_o.parameters(), lr=1e-3, weight_decay=1e-5)
    store = GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)
    hs = [BatchHandle(store, np.array(b)) for b in batches]
    step = FusedTrainStep(model)
    lo, lg = [], []
    for s in range(40):
        bat = P.Batch.from_data_list([datas[i].clone() for i in batches[s % 4]])
        opt_o.zero_grad()
        loss_o = torch.nn.functional.mse_loss(model_o(bat).reshape(-1), bat.y)
        loss_o.backward()
        opt_o.step()
        lo.append(float(loss_o.detach()))
        loss, _ = step.step(hs[s % 4])
        lg.append(float(loss))
    assert lo[0] > 100 * lo[-1]  # the large-initial-loss regime of the bench
    np.testing.assert_allclose(lg, lo, rtol=2e-3)
    ref = dict(model_o.named_parameters())
    for n, p in zip(amd.PARAM_NAMES, step.params):
        np.testing.assert_allclose(p.detach().cpu().numpy(), ref[n].detach().numpy(), rtol=2e-3, atol=2e-4, err_msg=n)
