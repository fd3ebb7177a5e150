"""Pin the CPU oracle against golden vectors produced by the reference itself.

The golden fixtures come from importing ``/root/reference/deeprank2`` modules
(``tests/golden/make_golden.py``); these tests need neither the reference nor a GPU.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch
from _util import assert_grad_close, fixed_dropout, golden_batch, golden_grads, golden_state_dict

from oracle import gnn_ref
from oracle import pyg_ops as P

TOL = dict(rtol=1e-5, atol=1e-5)


def _run(model, z, loss_kind, mask=None):
    model.load_state_dict(golden_state_dict(z))
    model.eval()
    with torch.no_grad():
        out_eval = model(golden_batch(z)).numpy()
    model.train()
    if mask is not None:
        model.dropout_fn = fixed_dropout(torch.from_numpy(mask))
    model.zero_grad()
    b = golden_batch(z)
    out = model(b)
    y = torch.from_numpy(z["in/y"])
    loss = torch.nn.functional.mse_loss(out.reshape(-1), y) if loss_kind == "mse" else torch.nn.functional.cross_entropy(out, y.long())
    loss.backward()
    grads = {n: (p.grad if p.grad is not None else torch.zeros_like(p)).numpy() for n, p in model.named_parameters()}
    return out_eval, out.detach().numpy(), float(loss.detach()), grads


@pytest.mark.parametrize("name,cls,args", [
    ("ginet_1atn", "GINet", (50, 1, 1)),
    ("ginet_synth_regress", "GINet", (30, 1, 3)),
    ("ginet_synth_classif", "GINet", (30, 2, 3)),
    ("foutnet_synth", "FoutNet", (30, 1)),
    ("vanilla_synth", "VanillaNetwork", (30, 1, 3)),
    ("vanilla_pretrained_testhdf5", "VanillaNetwork", (26, 2, 1)),  # the reference's pre-trained weights on test.hdf5
    ("sgat_1atn", "SGAT", (50, 1)),
    ("sgat_synth", "SGAT", (30, 2)),
    ("ginet_nocluster_1atn", "GINetNoCluster", (50, 1, 1)),
    ("ginet_nocluster_synth", "GINetNoCluster", (30, 3, 3)),
])
def test_model_matches_reference(golden, name, cls, args):
    z = golden(name)
    model = gnn_ref.MODELS[cls](*args)
    loss_kind = str(z["meta/loss"])
    out_eval, out_train, loss, grads = _run(model, z, loss_kind, z.get("mask"))
    np.testing.assert_allclose(out_eval, z["out/eval"], **TOL)
    np.testing.assert_allclose(out_train, z["out/train"], **TOL)
    assert loss == pytest.approx(float(z["loss"]), rel=1e-5, abs=1e-6)
    ref = golden_grads(z)
    assert set(ref) == set(grads)
    for k in ref:  # rtol 1e-4 plus a normwise floor: CPU thread counts change summation order
        assert_grad_close(grads[k], ref[k], err_msg=k)


@pytest.mark.parametrize("name,cls", [("ginet_nonfinite_all", "GINet"), ("ginet_nonfinite_conv1", "GINet"), ("ginet_nocluster_nonfinite", "GINetNoCluster")])
def test_model_matches_reference_nonfinite_inputs(golden, name, cls):
    """inf edge attributes / NaN node features: the reference's singleton
    softmax gives NaN for a non-finite logit (ginet.py:48-54); NaN outputs and
    gradients must sit exactly where the reference's are."""
    z = golden(name)
    out_eval, out_train, loss, grads = _run(gnn_ref.MODELS[cls](30, 1, 3), z, "mse", z["mask"])
    np.testing.assert_allclose(out_eval, z["out/eval"], **TOL)
    np.testing.assert_allclose(out_train, z["out/train"], **TOL)
    np.testing.assert_allclose(loss, float(z["loss"]), rtol=1e-5)
    ref = golden_grads(z)
    for k in ref:
        assert_grad_close(grads[k], ref[k], err_msg=k)


def test_conv_layer_nonfinite_edge_attr(golden):
    z = golden("ginet_conv_layer_nonfinite")
    layer = gnn_ref.GINetConvLayer(12, 16, 2)
    layer.load_state_dict(golden_state_dict(z))
    x = torch.from_numpy(z["in/x"]).requires_grad_(True)
    out = layer(x, torch.from_numpy(z["in/edge_index"]), torch.from_numpy(z["in/edge_attr"]))
    (out * torch.from_numpy(z["in/gz"])).sum().backward()
    np.testing.assert_allclose(out.detach().numpy(), z["out/z"], **TOL)
    np.testing.assert_allclose(x.grad.numpy(), z["grad/x"], **TOL)
    for n, p in layer.named_parameters():
        np.testing.assert_allclose(p.grad.numpy(), z["grad/" + n], **TOL, err_msg=n)


def test_ginet_dead_attention_grads_are_exactly_zero(golden):
    """softmax over the singleton dim makes the attention constant."""
    z = golden("ginet_1atn")
    for k, v in golden_grads(z).items():
        if "fc_attention" in k or "fc_edge_attr" in k:
            assert np.all(v == 0.0), k
            assert bool(z["hasgrad/" + k]), "reference gives a zero tensor, not None"


def test_ginet_batch1_equals_batch4(golden):
    z = golden("ginet_1atn")
    np.testing.assert_allclose(z["out/eval_b1"], z["out/eval"], rtol=2e-6, atol=1e-5)


def test_foutnet_testhdf5_nan(golden):
    """test.hdf5 has one depth-0 cluster per graph: the pooled conv sees no edges
    and FoutLayer's mean over an empty neighbour set is NaN (foutnet.py:58)."""
    z = golden("foutnet_testhdf5")
    model = gnn_ref.FoutNet(50, 2)
    model.load_state_dict(golden_state_dict(z))
    model.eval()
    with torch.no_grad():
        out = model(golden_batch(z)).numpy()
    assert np.isnan(z["out/eval"]).all()
    assert np.isnan(out).all()


def test_conv_layer_arbitrary_edges(golden):
    z = golden("ginet_conv_layer")
    layer = gnn_ref.GINetConvLayer(12, 16, 2)
    layer.load_state_dict(golden_state_dict(z))
    x = torch.from_numpy(z["in/x"]).requires_grad_(True)
    out = layer(x, torch.from_numpy(z["in/edge_index"]), torch.from_numpy(z["in/edge_attr"]))
    (out * torch.from_numpy(z["in/gz"])).sum().backward()
    np.testing.assert_allclose(out.detach().numpy(), z["out/z"], **TOL)
    np.testing.assert_allclose(x.grad.numpy(), z["grad/x"], **TOL)
    np.testing.assert_allclose(layer.fc.weight.grad.numpy(), z["grad/fc.weight"], rtol=1e-4, atol=1e-5)


def test_community_pooling(golden):
    z = golden("community_pooling_1atn")
    b = golden_batch(z)
    c = gnn_ref.offset_clusters_inplace(b.cluster0.clone(), b.batch)
    np.testing.assert_array_equal(c.numpy(), z["out/cluster_offset"])
    pooled = gnn_ref.pool_communities(c, b)
    np.testing.assert_array_equal(pooled.x.numpy(), z["out/x"])
    np.testing.assert_array_equal(pooled.edge_index.numpy(), z["out/edge_index"])
    np.testing.assert_allclose(pooled.edge_attr.numpy(), z["out/edge_attr"], rtol=1e-6)
    np.testing.assert_array_equal(pooled.batch.numpy(), z["out/batch"])


def test_scatter_max_semantics():
    """torch_scatter: NaN never wins, ties keep the first member, empty -> 0."""
    src = torch.tensor([[1.0], [float("nan")], [1.0], [0.5], [-2.0]])
    idx = torch.tensor([0, 0, 0, 2, 2])
    out, arg = P.scatter_max(src, idx, dim_size=4)
    assert out.view(-1).tolist() == [1.0, 0.0, 0.5, 0.0]
    assert arg.view(-1).tolist() == [0, 5, 3, 5]
    amax = P.pyg_scatter(src, idx, reduce="max")
    assert np.isnan(amax[0, 0].item())


@pytest.mark.parametrize("name", ["sgat_layer", "sgat_layer_directed"])
def test_sgat_layer_matches_reference(golden, name):
    z = golden(name)
    layer = gnn_ref.SGraphAttentionLayer(12, 16, undirected=bool(z["meta/undirected"]))
    layer.load_state_dict({k[6:]: torch.from_numpy(v) for k, v in z.items() if k.startswith("param/")})
    x = torch.from_numpy(z["in/x"]).requires_grad_(True)
    out = layer(x, torch.from_numpy(z["in/edge_index"]), torch.from_numpy(z["in/edge_attr"]))
    (out * torch.from_numpy(z["in/gz"])).sum().backward()
    np.testing.assert_allclose(out.detach().numpy(), z["out/z"], **TOL)
    np.testing.assert_allclose(x.grad.numpy(), z["grad/x"], rtol=1e-4, atol=1e-5)
    for n, p in layer.named_parameters():
        np.testing.assert_allclose(p.grad.numpy(), z["grad/" + n], rtol=1e-4, atol=1e-5, err_msg=n)
