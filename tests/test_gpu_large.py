"""Large-graph GINet path (dr_ginet_large_pass: per-tile conv1 kernel + per-graph
tail) — config 4's atom-level graphs (N ~ 3e3, E ~ 5e4) do not fit one
workgroup's LDS.

* On residue graphs forced through it, it is bit-identical to the
  single-workgroup kernel (same gather order, same MFMA chain, same tail).
* On atom-level graphs it matches the CPU oracle (module autograd and the
  fused train step + Adam).  Tolerance: 1e-4 (north_star, fp32).
"""

from __future__ import annotations

import numpy as np
import pytest
import torch
from _util import assert_grad_close

from deeprank2_amd import _lib
from deeprank2_amd.engine import FusedTrainStep
from deeprank2_amd.fused import BatchHandle, Dropout
from deeprank2_amd.neuralnets.gnn import ginet as amd
from deeprank2_amd.store import GraphStore, pack_graphs, records_from_batch
from deeprank2_amd.utils.synthetic import make_dataset
from oracle import data_ref, gnn_ref
from oracle import pyg_ops as P

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = dict(rtol=1e-4, atol=1e-4)


def _datas(n, seed, **kw):
    return [data_ref.synthetic_to_data(g, f"g{i}") for i, g in enumerate(make_dataset(n, seed=seed, **kw))]


def _atoms(n, seed):
    ds = _datas(n, seed, n_lo=2700, n_hi=3300, mean_degree=16.7, k_lo=8, k_hi=32)
    for i, d in enumerate(ds):  # several depth-1 clusters on some graphs
        k = len(d.cluster1)
        if i % 2:
            d.cluster1 = torch.tensor([j % 3 for j in range(k)], dtype=torch.long)
    return ds


def _store(datas):
    return GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)


def test_large_path_bit_identical_to_single_workgroup_kernel():
    datas = _datas(16, seed=21)
    store = _store(datas)
    torch.manual_seed(3)
    model = amd.GINet(30, 2, 3).to(DEV)
    params = model.ordered_params()
    res = []
    for force, halos, amax in ((False, True, True), (True, True, True), (True, False, True), (True, True, False), (True, False, False)):
        h = BatchHandle(store, np.arange(16))
        h.force_large = force
        h.large_halos = halos
        h.large_atomic_max = amax
        out = torch.empty(16, 2, device=DEV)
        slab = torch.empty(16 * amd.slab_stride(30), device=DEV)
        head = torch.zeros(16 * amd.head_stride(2), device=DEV)
        lpg = torch.empty(16, device=DEV)
        store.set_targets(np.arange(16) % 2)
        amd.graph_pass(h, params, 2, 3, loss_kind=_lib.DR_LOSS_CE, loss_scale=1 / 16, dropout=Dropout(0.4, seed=7, offset=3), out=out, loss_per_graph=lpg, slab=slab, head=head)
        torch.cuda.synchronize()
        res.append((out.cpu(), slab.cpu(), head.cpu(), lpg.cpu()))
    for other in res[1:]:  # split path with tile halos in LDS, and with the per-edge HBM gather
        for x, y in zip(res[0], other):
            assert torch.equal(x, y)


def test_atom_graphs_halo_and_hbm_gather_bit_identical():
    store = _store(_atoms(3, seed=5))
    torch.manual_seed(4)
    model = amd.GINet(30, 1, 3).to(DEV)
    params = model.ordered_params()
    res = []
    for halos, amax in ((True, True), (False, False), (True, False)):
        h = BatchHandle(store, np.arange(3))
        h.large_halos = halos
        h.large_atomic_max = amax
        assert (h.large_plan(1).halo_tensors is not None) == halos
        out = torch.empty(3, 1, device=DEV)
        slab = torch.empty(3 * amd.slab_stride(30), device=DEV)
        head = torch.zeros(3 * amd.head_stride(1), device=DEV)
        amd.graph_pass(h, params, 1, 3, loss_kind=_lib.DR_LOSS_MSE, loss_scale=1 / 3, out=out, slab=slab, head=head)
        torch.cuda.synchronize()
        res.append((out.cpu(), slab.cpu(), head.cpu()))
    for other in res[1:]:
        for x, y in zip(res[0], other):
            assert torch.equal(x, y)


def test_atom_graphs_module_vs_oracle():
    datas = _atoms(3, seed=5)
    assert max(d.x.shape[0] for d in datas) > 2600 and max(d.edge_index.shape[1] for d in datas) > 40000
    torch.manual_seed(9)
    model_o = gnn_ref.GINet(30, 1, 3).eval()
    model = amd.GINet(30, 1, 3)
    model.load_state_dict(model_o.state_dict())
    model = model.to(DEV).eval()
    out_o = model_o(P.Batch.from_data_list([d.clone() for d in datas]))
    (out_o.square().sum()).backward()
    b = P.Batch.from_data_list(datas)
    out = model(b)
    out.square().sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), out_o.detach().numpy(), **TOL)
    ref = dict(model_o.named_parameters())
    for n, p in model.named_parameters():
        assert_grad_close(p.grad.cpu().numpy(), ref[n].grad.numpy(), err_msg=n)


def test_atom_graphs_fused_train_step_vs_oracle():
    datas = _atoms(4, seed=6)
    torch.manual_seed(10)
    model_o = gnn_ref.GINet(30, 1, 3)
    model = amd.GINet(30, 1, 3)
    model.load_state_dict(model_o.state_dict())
    model = model.to(DEV).train()
    mask = (torch.rand(4, 128, generator=torch.Generator().manual_seed(1)) >= 0.4).float()
    model_o.train()
    from _util import fixed_dropout

    model_o.dropout_fn = fixed_dropout(mask)
    bat = P.Batch.from_data_list([d.clone() for d in datas])
    out_o = model_o(bat)
    loss_o = torch.nn.functional.mse_loss(out_o.reshape(-1), bat.y)
    loss_o.backward()
    h = BatchHandle(_store(datas), np.arange(4))
    assert h.lds(("dr_ginet_graph_pass", 1), lambda *s: _lib.load().dr_ginet_lds_bytes(s[0], s[1], 30, s[2], s[3], s[4], 1, 1)) > 160 * 1024
    step = FusedTrainStep(model)
    loss, out = step.step(h, mask=mask.to(torch.uint8).to(DEV))
    np.testing.assert_allclose(out.cpu().numpy(), out_o.detach().numpy(), **TOL)
    assert float(loss) == pytest.approx(float(loss_o.detach()), rel=1e-4)
    grads = dict(zip(amd.PARAM_NAMES, step.grads))
    for n, p in model_o.named_parameters():
        assert_grad_close(grads[n].cpu().numpy(), p.grad.numpy(), err_msg=n)
