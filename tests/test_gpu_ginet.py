"""GPU parity of the MI355X GINet path (HIP kernels via the C ABI) against the
reference goldens and the CPU oracle.  Tolerance: 1e-4 (north_star, fp32)."""

from __future__ import annotations

import numpy as np
import pytest
import torch
from _util import assert_grad_close, fixed_dropout, golden_batch, golden_graphs, golden_grads, golden_state_dict

from deeprank2_amd.engine import GINetTrainStep
from deeprank2_amd.neuralnets.gnn import ginet as amd
from deeprank2_amd.store import GraphStore, pack_graphs, records_from_batch
from oracle import data_ref, gnn_ref
from oracle import pyg_ops as P

pytestmark = pytest.mark.gpu
TOL = dict(rtol=1e-4, atol=1e-4)
DEV = "cuda:0"


def _model(z, cls_args):
    m = amd.GINet(*cls_args)
    m.load_state_dict(golden_state_dict(z))
    return m.to(DEV)


@pytest.mark.parametrize("name,args", [("ginet_1atn", (50, 1, 1)), ("ginet_synth_regress", (30, 1, 3)), ("ginet_synth_classif", (30, 2, 3))])
def test_ginet_module_vs_reference_golden(golden, name, args):
    z = golden(name)
    m = _model(z, args)
    m.eval()
    with torch.no_grad():
        out = m(golden_batch(z)).cpu().numpy()
    np.testing.assert_allclose(out, z["out/eval"], **TOL)

    m.train()
    m.zero_grad()
    out = m(golden_batch(z), dropout_mask=torch.from_numpy(z["mask"]).to(torch.uint8))
    y = torch.from_numpy(z["in/y"]).to(DEV)
    loss = torch.nn.functional.mse_loss(out.reshape(-1), y) if str(z["meta/loss"]) == "mse" else torch.nn.functional.cross_entropy(out, y.long())
    loss.backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), z["out/train"], **TOL)
    assert float(loss.detach()) == pytest.approx(float(z["loss"]), rel=1e-4)
    ref = golden_grads(z)
    for n, p in m.named_parameters():
        assert p.grad is not None, n
        assert_grad_close(p.grad.cpu().numpy(), ref[n], err_msg=n)


def test_ginet_batch1_hip_vs_reference_golden(golden):
    """configs[0]: the reference's 1ATN fixture, one graph per batch (the
    reference CPU Trainer's batch_size=1), each graph through the HIP pass
    against the reference's own batch-1 outputs (``out/eval_b1``)."""
    z = golden("ginet_1atn")
    m = _model(z, (50, 1, 1)).eval()
    ptr = np.asarray(z["in/ptr"])
    ei = np.asarray(z["in/edge_index"])
    ref_b1 = np.asarray(z["out/eval_b1"]).reshape(ptr.size - 1, -1)
    for g, (_, n, c0, c1) in enumerate(golden_graphs(z)):
        lo, hi = int(ptr[g]), int(ptr[g + 1])
        em = (ei[0] >= lo) & (ei[0] < hi)
        d = P.Data(
            x=torch.from_numpy(np.array(z["in/x"][lo:hi])),
            edge_index=torch.from_numpy(ei[:, em] - lo),
            edge_attr=torch.from_numpy(np.array(z["in/edge_attr"])[em]),
            cluster0=torch.from_numpy(np.array(c0)),
            cluster1=torch.from_numpy(np.array(c1)),
            y=torch.from_numpy(np.array(z["in/y"])[g : g + 1]),
        )
        assert d.x.shape[0] == n
        with torch.no_grad():
            out = m(P.Batch.from_data_list([d])).cpu().numpy()
        np.testing.assert_allclose(out.reshape(-1), ref_b1[g], **TOL, err_msg=f"graph {g}")


def test_conv_layer_arbitrary_edges_vs_golden(golden):
    z = golden("ginet_conv_layer")
    layer = amd.GINetConvLayer(12, 16, 2)
    layer.load_state_dict(golden_state_dict(z))
    layer = layer.to(DEV)
    x = torch.from_numpy(z["in/x"]).to(DEV).requires_grad_(True)
    out = layer(x, torch.from_numpy(z["in/edge_index"]).to(DEV), torch.from_numpy(z["in/edge_attr"]).to(DEV))
    (out * torch.from_numpy(z["in/gz"]).to(DEV)).sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), z["out/z"], **TOL)
    np.testing.assert_allclose(x.grad.cpu().numpy(), z["grad/x"], **TOL)
    np.testing.assert_allclose(layer.fc.weight.grad.cpu().numpy(), z["grad/fc.weight"], **TOL)
    assert torch.count_nonzero(layer.fc_attention.weight.grad) == 0


def _synthetic(n, seed, **kw):
    from deeprank2_amd.utils.synthetic import make_dataset

    return [data_ref.synthetic_to_data(g, f"s{i}") for i, g in enumerate(make_dataset(n, seed=seed, **kw))]


def _oracle_step(model_o, datas, mask):
    model_o.train()
    model_o.dropout_fn = fixed_dropout(mask)
    model_o.zero_grad()
    bat = P.Batch.from_data_list(datas)
    out = model_o(bat)
    loss = torch.nn.functional.mse_loss(out.reshape(-1), bat.y)
    loss.backward()
    return out.detach().numpy(), float(loss.detach())


def test_fused_train_step_vs_oracle_config2_batch64():
    """Config 2 shape (B=64 synthetic residue graphs, F=30, Fe=3): fused
    fwd+loss+bwd kernel + reduce/Adam against the oracle + torch.optim.Adam."""
    torch.manual_seed(1234)
    datas = _synthetic(64, seed=0)
    model_o = gnn_ref.GINet(30, 1, 3)
    model = amd.GINet(30, 1, 3)
    model.load_state_dict(model_o.state_dict())
    model = model.to(DEV).train()
    mask = (torch.rand(64, 128, generator=torch.Generator().manual_seed(3)) >= 0.4).float()
    out_o, loss_o = _oracle_step(model_o, [d.clone() for d in datas], mask)

    store = GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)
    h = amd.BatchHandle(store, np.arange(64))
    step = GINetTrainStep(model)
    before = [p.detach().clone() for p in step.params]
    loss, out = step.step(h, mask=mask.to(torch.uint8).to(DEV))
    np.testing.assert_allclose(out.cpu().numpy(), out_o, **TOL)
    assert float(loss) == pytest.approx(loss_o, rel=1e-4)
    grads = dict(zip(amd.PARAM_NAMES, step.grads))
    for n, p in model_o.named_parameters():
        assert_grad_close(grads[n].cpu().numpy(), p.grad.numpy(), err_msg=n)
    # the fused Adam against torch.optim.Adam fed the same (kernel) gradients
    ref = [torch.nn.Parameter(b) for b in before]
    for r, g in zip(ref, step.grads):
        r.grad = g.detach().clone()
    torch.optim.Adam(ref, lr=1e-3, weight_decay=1e-5).step()
    for n, r, p in zip(amd.PARAM_NAMES, ref, step.params):
        np.testing.assert_allclose(p.detach().cpu().numpy(), r.detach().cpu().numpy(), rtol=1e-5, atol=1e-7, err_msg=n)


@pytest.mark.parametrize("f", [12, 40])
def test_fused_train_step_vs_oracle_other_feature_counts(f):
    """F = 12 (K padded to 16 under the 32-wide kernel) and F = 40 (48 under
    the 64-wide kernel): the per-graph kernel's Z rows are shorter than the
    kernel's K there.  (Before r05 the Z padding was zeroed to the kernel's
    K, 14 words past Z into the row pointers DMA'd beside it: wrong outputs
    whenever the zeroing landed after the DMA.)  Five launches, each against
    the oracle."""
    torch.manual_seed(1234)
    datas = _synthetic(16, seed=5, n_feat=f)
    model_o = gnn_ref.GINet(f, 1, 3)
    mask = (torch.rand(16, 128, generator=torch.Generator().manual_seed(3)) >= 0.4).float()
    out_o, loss_o = _oracle_step(model_o, [d.clone() for d in datas], mask)
    store = GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)
    h = amd.BatchHandle(store, np.arange(16))
    for _ in range(5):
        model = amd.GINet(f, 1, 3)
        model.load_state_dict(model_o.state_dict())
        step = GINetTrainStep(model.to(DEV).train())
        loss, out = step.step(h, mask=mask.to(torch.uint8).to(DEV))
        np.testing.assert_allclose(out.cpu().numpy(), out_o, **TOL)
        assert float(loss) == pytest.approx(loss_o, rel=1e-4)


def test_module_autograd_vs_oracle_single_cluster_graphs():
    """test.hdf5-like batches: one depth-0 cluster per graph -> conv2 sees no
    edges; also a graph with several depth-1 clusters."""
    datas = _synthetic(6, seed=11, n_lo=30, n_hi=60, mean_degree=8.0)
    for d in datas[:3]:
        d.cluster0 = torch.zeros_like(d.cluster0)
        d.cluster1 = torch.zeros(1, dtype=torch.long)
    torch.manual_seed(7)
    model_o = gnn_ref.GINet(30, 1, 3).eval()
    model = amd.GINet(30, 1, 3)
    model.load_state_dict(model_o.state_dict())
    model = model.to(DEV).eval()
    out_o = model_o(P.Batch.from_data_list([d.clone() for d in datas]))
    loss_o = out_o.square().sum()
    loss_o.backward()
    out = model(P.Batch.from_data_list(datas))
    out.square().sum().backward()
    np.testing.assert_allclose(out.detach().cpu().numpy(), out_o.detach().numpy(), **TOL)
    ref = dict(model_o.named_parameters())
    for n, p in model.named_parameters():
        assert_grad_close(p.grad.cpu().numpy(), ref[n].grad.numpy(), err_msg=n)


def test_deterministic_bitwise():
    datas = _synthetic(16, seed=4)
    store = GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)
    h = amd.BatchHandle(store, np.arange(16))
    torch.manual_seed(0)
    model = amd.GINet(30, 1, 3).to(DEV)
    params = model.ordered_params()
    outs = []
    for _ in range(3):
        slab = torch.empty(16 * amd.slab_stride(30), device=DEV)
        head = torch.empty(16 * amd.head_stride(1), device=DEV)
        out = torch.empty(16, 1, device=DEV)
        amd.graph_pass(h, params, 1, 3, loss_kind=1, loss_scale=1 / 16, out=out, loss_per_graph=torch.empty(16, device=DEV), slab=slab, head=head)
        outs.append((out.cpu(), slab.cpu()))
    for o, s in outs[1:]:
        assert torch.equal(o, outs[0][0])
        assert torch.equal(s, outs[0][1])


def test_gids_subset_and_permutation():
    """A mini-batch is a list of graph ids into the resident store: any order/subset."""
    datas = _synthetic(10, seed=6)
    store = GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)
    torch.manual_seed(1)
    model_o = gnn_ref.GINet(30, 1, 3).eval()
    model = amd.GINet(30, 1, 3)
    model.load_state_dict(model_o.state_dict())
    model = model.to(DEV).eval()
    gids = np.array([7, 2, 9, 0])
    b = P.Batch.from_data_list([datas[i].clone() for i in gids])
    b._dr_handle = amd.BatchHandle(store, gids)
    with torch.no_grad():
        out = model(b).cpu().numpy()
        ref = model_o(P.Batch.from_data_list([datas[i].clone() for i in gids])).numpy()
    np.testing.assert_allclose(out, ref, **TOL)


def test_cpu_model_raises():
    m = amd.GINet(30, 1, 3)
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        m(P.Batch.from_data_list(_synthetic(1, seed=1)))


def test_hash_dropout_matches_host_replica_mask():
    """In-kernel dropout RNG (DR_DROPOUT_HASH) == the same keep mask fed explicitly."""
    from deeprank2_amd import _lib

    datas = _synthetic(12, seed=9)
    store = GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)
    h = amd.BatchHandle(store, np.arange(12))
    torch.manual_seed(2)
    model = amd.GINet(30, 1, 3).to(DEV)
    params = model.ordered_params()
    outs = []
    keep = torch.from_numpy(_lib.dropout_keep_host(99, 5, 12 * 128, 0.4).reshape(12, 128)).to(DEV)
    for drop in (amd.Dropout(0.4, seed=99, offset=5), amd.Dropout(0.4, mask=keep)):
        out = torch.empty(12, 1, device=DEV)
        slab = torch.empty(12 * amd.slab_stride(30), device=DEV)
        head = torch.zeros(12 * amd.head_stride(1), device=DEV)
        amd.graph_pass(h, params, 1, 3, dropout=drop, loss_kind=1, loss_scale=1 / 12, out=out, loss_per_graph=torch.empty(12, device=DEV), slab=slab, head=head)
        outs.append((out.cpu(), slab.cpu(), head.cpu()))
    for x, y in zip(*outs):
        assert torch.equal(x, y)


def test_captured_step_replay_matches_eager():
    """hipGraph replay of the fused step == eager steps (device step counter
    advances dropout offset and Adam's step on every replay)."""
    datas = _synthetic(32, seed=12)
    store = GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)
    hs = [amd.BatchHandle(store, np.arange(16)), amd.BatchHandle(store, np.arange(16, 32))]
    torch.manual_seed(3)
    m1 = amd.GINet(30, 1, 3).to(DEV).train()
    m2 = amd.GINet(30, 1, 3).to(DEV).train()
    m2.load_state_dict(m1.state_dict())
    m1._drop_seed = m2._drop_seed = 1234
    s1, s2 = GINetTrainStep(m1), GINetTrainStep(m2)
    graphs = [s2.capture(h) for h in hs]
    for i in range(6):
        l1, _ = s1.step(hs[i % 2])
        graphs[i % 2].replay()
        torch.cuda.synchronize()
        assert torch.equal(l1, s2.loss_out), i
    for a, b in zip(s1.params, s2.params):
        assert torch.equal(a, b)
    assert int(s1.counter[0]) == int(s2.counter[0]) == 6


def test_captured_sweep_matches_eager():
    """One HIP graph holding a sweep of steps over several mini-batches == eager steps."""
    datas = _synthetic(36, seed=13)
    store = GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)
    hs = [amd.BatchHandle(store, np.arange(12 * k, 12 * k + 12)) for k in range(3)]
    torch.manual_seed(5)
    m1 = amd.GINet(30, 1, 3).to(DEV).train()
    m2 = amd.GINet(30, 1, 3).to(DEV).train()
    m2.load_state_dict(m1.state_dict())
    m1._drop_seed = m2._drop_seed = 99
    s1, s2 = GINetTrainStep(m1), GINetTrainStep(m2)
    sweep = s2.capture_sweep(hs)
    for _ in range(2):
        for h in hs:
            l1, _ = s1.step(h)
        sweep.replay()
    torch.cuda.synchronize()
    assert torch.equal(l1, s2.loss_out)
    for a, b in zip(s1.params, s2.params):
        assert torch.equal(a, b)
    assert int(s2.counter[0]) == 6


def test_accumulating_pass_vs_oracle_batch300():
    """a batch past the CU count (B = 300) takes the
    accumulating pass by default (``FusedTrainStep.acc = None``:
    ``dr_ginet_acc_pass``, each workgroup summing its graphs' gradients on
    chip).  Outputs, loss and every gradient against the oracle
    (``ginet.py:90-125`` under ``trainer.py:686-690``), then one fused Adam
    step against torch.optim.Adam, as the B = 64 test above."""
    torch.manual_seed(4321)
    datas = _synthetic(300, seed=21)
    model_o = gnn_ref.GINet(30, 1, 3)
    model = amd.GINet(30, 1, 3)
    model.load_state_dict(model_o.state_dict())
    model = model.to(DEV).train()
    mask = (torch.rand(300, 128, generator=torch.Generator().manual_seed(8)) >= 0.4).float()
    out_o, loss_o = _oracle_step(model_o, [d.clone() for d in datas], mask)

    store = GraphStore(pack_graphs(records_from_batch(P.Batch.from_data_list(datas))), DEV)
    h = amd.BatchHandle(store, np.arange(300))
    step = GINetTrainStep(model)
    assert step.acc is None and step._acc_rows(h) > 0  # noqa: SLF001  (the default path is the accumulating pass)
    before = [p.detach().clone() for p in step.params]
    loss, out = step.step(h, mask=mask.to(torch.uint8).to(DEV))
    np.testing.assert_allclose(out.cpu().numpy(), out_o, **TOL)
    assert float(loss) == pytest.approx(loss_o, rel=1e-4)
    grads = dict(zip(amd.PARAM_NAMES, step.grads))
    for n, p in model_o.named_parameters():
        assert_grad_close(grads[n].cpu().numpy(), p.grad.numpy(), err_msg=n)
    ref = [torch.nn.Parameter(b) for b in before]
    for r, g in zip(ref, step.grads):
        r.grad = g.detach().clone()
    torch.optim.Adam(ref, lr=1e-3, weight_decay=1e-5).step()
    for n, r, p in zip(amd.PARAM_NAMES, ref, step.params):
        np.testing.assert_allclose(p.detach().cpu().numpy(), r.detach().cpu().numpy(), rtol=1e-5, atol=1e-7, err_msg=n)
