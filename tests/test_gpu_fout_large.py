"""Large-graph FoutNet / SGAT path (dr_fout_large_pass / dr_sgat_large_pass:
per-tile conv1 kernel + per-graph tail) for graphs beyond one workgroup's LDS
(atom level, BASELINE configs[4]'s 20 %).

* On residue graphs forced through it, it is bit-identical to the
  single-workgroup kernels (same gather order, same MFMA chain, same pool
  decisions, same tail), with and without LDS halos, including the NaN rows
  of nodes without out-edges (FoutLayer's torch.mean(empty)).
* On atom-level graphs it matches the CPU oracle (forward, loss, every
  gradient) and the fused training step runs it.  Tolerance: 1e-4
  (north_star, fp32) with tests/_util.py's normwise gradient floor.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch
from _util import assert_grad_close

from deeprank2_amd import _lib, layered
from deeprank2_amd.engine import FusedTrainStep
from deeprank2_amd.fused import BatchHandle, LDS_MAX, lds_for
from deeprank2_amd.neuralnets.gnn import foutnet, sgat
from deeprank2_amd.store import GraphStore, pack_graphs, records_from_batch
from deeprank2_amd.utils.synthetic import make_dataset
from oracle import data_ref, gnn_ref
from oracle import pyg_ops as P

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = dict(rtol=1e-4, atol=1e-4)
MODELS = {"foutnet": (foutnet, gnn_ref.FoutNet, 3), "sgat": (sgat, gnn_ref.SGAT, 1)}


def _datas(n, seed, fe, **kw):
    out = []
    for i, g in enumerate(make_dataset(n, seed=seed, **kw)):
        d = data_ref.synthetic_to_data(g, f"f{i}")
        d.edge_attr = d.edge_attr[:, :fe].contiguous()
        out.append(d)
    return out


def _drop_out_edges(d, node):
    """Node `node` keeps its in-edges but has no out-edge (a NaN row in FoutNet)."""
    d.edge_index, d.edge_attr = d.edge_index[:, d.edge_index[0] != node], d.edge_attr[d.edge_index[0] != node]
    return d


def _store(datas):
    return GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)


@pytest.mark.parametrize("name", ["foutnet", "sgat"])
def test_large_path_bit_identical_to_single_workgroup_kernel(name):
    mod, _, fe = MODELS[name]
    datas = _datas(12, seed=31, fe=fe)
    if name == "foutnet":
        _drop_out_edges(datas[2], 7)
        _drop_out_edges(datas[5], 0)
    store = _store(datas)
    torch.manual_seed(5)
    model = (foutnet.FoutNet if name == "foutnet" else sgat.SGAT)(30, 2, fe).to(DEV)
    params = model.ordered_params()
    res = []
    for force, halos in ((False, True), (True, True), (True, False)):
        h = BatchHandle(store, np.arange(12))
        h.force_large, h.large_halos = force, halos
        out = torch.empty(12, 2, device=DEV)
        slab = torch.empty(12 * foutnet.slab_stride(30), device=DEV)  # SGAT shares FoutNet's partial layout
        head = torch.zeros(12 * foutnet.head_stride(2), device=DEV)
        lpg = torch.empty(12, device=DEV)
        store.set_targets(np.arange(12) % 2)
        mod.graph_pass(h, params, 2, 3, loss_kind=_lib.DR_LOSS_CE, loss_scale=1 / 12, out=out, loss_per_graph=lpg, slab=slab, head=head)
        torch.cuda.synchronize()
        res.append((out.cpu(), slab.cpu(), head.cpu(), lpg.cpu()))
    for other in res[1:]:
        for x, y in zip(res[0], other):
            assert torch.equal(x, y)


@pytest.mark.parametrize("name", ["foutnet", "sgat"])
def test_atom_graphs_module_vs_oracle(name):
    mod, ref_cls, fe = MODELS[name]
    datas = _datas(2, seed=33, fe=fe, n_lo=2600, n_hi=3000, mean_degree=16.0, k_lo=8, k_hi=20)
    torch.manual_seed(6)
    model_o = ref_cls(30, 1, fe)
    model = (foutnet.FoutNet if name == "foutnet" else sgat.SGAT)(30, 1, fe)
    model.load_state_dict(model_o.state_dict())
    model = model.to(DEV).train()
    bat = P.Batch.from_data_list([d.clone() for d in datas])
    out_o = model_o(bat)
    loss_o = torch.nn.functional.mse_loss(out_o.reshape(-1), bat.y)
    loss_o.backward()
    store = _store(datas)
    h = BatchHandle(store, np.arange(2))
    assert lds_for(mod.SPEC, h, 1) > LDS_MAX and not layered.needs_layers(mod.SPEC, h, 1)
    from types import SimpleNamespace

    out = model(SimpleNamespace(_dr_handle=h))
    loss = torch.nn.functional.mse_loss(out.reshape(-1), torch.tensor([d.y.item() for d in datas], device=DEV))
    loss.backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), out_o.detach().numpy(), **TOL)
    assert float(loss.detach()) == pytest.approx(float(loss_o), rel=1e-4)
    ref = dict(model_o.named_parameters())
    for n, p in model.named_parameters():
        assert_grad_close(p.grad.cpu().numpy(), ref[n].grad.numpy(), err_msg=n)


def test_mixed_batch_fused_train_step_vs_oracle():
    """configs[4]'s mix (residue / SRV / atom graphs) through FusedTrainStep:
    loss and every gradient vs the oracle, then Adam as torch's."""
    datas = _datas(3, seed=35, fe=3) + _datas(2, seed=38, fe=3, n_lo=26, n_hi=36, mean_degree=7.0, k_lo=2, k_hi=3) + _datas(1, seed=37, fe=3, n_lo=2600, n_hi=2900, mean_degree=16.0, k_lo=8, k_hi=20)
    torch.manual_seed(7)
    model_o = gnn_ref.FoutNet(30, 1)
    model = foutnet.FoutNet(30, 1)
    model.load_state_dict(model_o.state_dict())
    bat = P.Batch.from_data_list([d.clone() for d in datas])
    loss_o = torch.nn.functional.mse_loss(model_o(bat).reshape(-1), bat.y)
    loss_o.backward()
    step = FusedTrainStep(model.to(DEV).train())
    h = BatchHandle(_store(datas), np.arange(len(datas)))
    loss, _ = step.step(h)
    assert float(loss) == pytest.approx(float(loss_o), rel=1e-4)
    ref = dict(model_o.named_parameters())
    for n, g in zip(foutnet.PARAM_NAMES, step.grads):
        assert_grad_close(g.cpu().numpy(), ref[n].grad.numpy(), err_msg=n)
