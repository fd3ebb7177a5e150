"""Host-side packing (GraphStore) and the fused kernel's algorithm, on CPU.

``ginet_store_model`` walks the packed store exactly like ``ginet_fused.hip``;
checking it against the reference goldens validates the packing and the
algebra (alpha == 1, fused branches, precomputed pooling, tie-splitting and
arg-member backward) without a GPU.
"""

from __future__ import annotations

import numpy as np
import pytest
import torch
from _util import golden_batch, golden_grads, golden_state_dict

import ginet_store_model as M
from deeprank2_amd.neuralnets.gnn.ginet import PARAM_NAMES
from deeprank2_amd.store import pack_graphs, records_from_batch
from oracle import gnn_ref


def _packed(z, y_override=None):
    recs = records_from_batch(golden_batch(z))
    if y_override is not None:
        for r, v in zip(recs, y_override):
            r.y = v
    return pack_graphs(recs)


def _params(z):
    sd = golden_state_dict(z)
    return [sd[n].numpy() for n in PARAM_NAMES]


@pytest.mark.parametrize("name", ["ginet_1atn", "ginet_synth_regress", "ginet_synth_classif"])
def test_store_model_matches_reference(golden, name):
    z = golden(name)
    out_dim = int(z["meta/out"])
    loss = str(z["meta/loss"])
    packed = _packed(z)
    params = _params(z)
    out_eval, _, _ = M.run(packed, params, out_dim, loss=loss)
    np.testing.assert_allclose(out_eval, z["out/eval"], rtol=1e-5, atol=1e-5)
    out, grads, lval = M.run(packed, params, out_dim, mask=z["mask"], drop_scale=1 / 0.6, loss=loss)
    np.testing.assert_allclose(out, z["out/train"], rtol=1e-5, atol=1e-5)
    assert lval == pytest.approx(float(z["loss"]), rel=1e-5)
    ref = golden_grads(z)
    for i, n in enumerate(PARAM_NAMES):
        np.testing.assert_allclose(grads[i], ref[n], rtol=1e-4, atol=2e-5, err_msg=n)


def test_pooled_graph_matches_community_pooling(golden):
    """The precomputed pooled CSR == pool_edge's coalesced edges (offset per graph)."""
    z = golden("community_pooling_1atn")
    packed = _packed(z)
    rows, cols = [], []
    for g in range(packed.n_graphs):
        k0a, k0b = packed.k0_off[g], packed.k0_off[g + 1]
        rp = packed.p1_rowptr[k0a + g:k0b + g + 1]
        q0 = packed.p1_off[g]
        for k in range(k0b - k0a):
            for e in range(rp[k], rp[k + 1]):
                rows.append(k0a + k)
                cols.append(k0a + packed.p1_col[q0 + e])
    np.testing.assert_array_equal(np.array([rows, cols]), z["out/edge_index"])
    # pooled edge_attr == pool_edge's coalesced sums (same slot order; the
    # summation order of merged edges follows torch.sort, so ulp-level only)
    np.testing.assert_allclose(packed.p1_ea, z["out/edge_attr"], rtol=1e-6)
    # transposed pooled slot -> pooled slot of the reversed edge
    for g in range(packed.n_graphs):
        k0a, k0b = packed.k0_off[g], packed.k0_off[g + 1]
        rp, trp = packed.p1_rowptr[k0a + g:k0b + g + 1], packed.p1t_rowptr[k0a + g:k0b + g + 1]
        q0 = packed.p1_off[g]
        row_of = np.repeat(np.arange(k0b - k0a), np.diff(rp))
        for b in range(k0b - k0a):
            for s in range(trp[b], trp[b + 1]):
                q = packed.p1t_pid[q0 + s]
                assert row_of[q] == packed.p1t_col[q0 + s] and packed.p1_col[q0 + q] == b
    # depth-0 dense ids == consecutive_cluster of the offset ids
    dense = np.concatenate([packed.cl0[packed.node_off[g]:packed.node_off[g + 1]] + packed.k0_off[g] for g in range(packed.n_graphs)])
    np.testing.assert_array_equal(dense, np.unique(z["out/cluster_offset"], return_inverse=True)[1])


def test_store_is_symmetric_for_doubled_edges(golden):
    packed = _packed(golden("ginet_1atn"))
    assert packed.transpose_aliased


def test_store_asymmetric_keeps_transpose():
    rec = records_from_batch(golden_batch({"in/x": np.zeros((4, 3), np.float32), "in/edge_index": np.array([[0, 1, 2], [1, 2, 3]]), "in/batch": np.zeros(4, np.int64), "in/cluster0": np.array([0, 0, 1, 1]), "in/cluster1": np.array([0, 0])}))
    p = pack_graphs(rec)
    assert not p.transpose_aliased
    assert p.rowptr.tolist() == [0, 1, 2, 3, 3]
    assert p.t_rowptr.tolist() == [0, 0, 1, 2, 3]
    assert p.t_col.tolist() == [0, 1, 2]


def test_pack_rejects_bad_clusters():
    rec = records_from_batch(golden_batch({"in/x": np.zeros((3, 2), np.float32), "in/edge_index": np.array([[0, 1], [1, 0]]), "in/batch": np.zeros(3, np.int64), "in/cluster0": np.array([0, 0, 1]), "in/cluster1": np.array([0, 0])}))
    rec[0].cluster1 = np.array([0, 0, 0])
    with pytest.raises(ValueError, match="cluster1"):
        pack_graphs(rec)


def test_store_model_vs_oracle_random_ties():
    """Integer-valued features force exact ties in both max-poolings."""
    from deeprank2_amd.utils.synthetic import make_dataset
    from oracle import data_ref
    from oracle import pyg_ops as P

    graphs = make_dataset(3, seed=5, n_lo=20, n_hi=30, mean_degree=6.0)
    datas = [data_ref.synthetic_to_data(g) for g in graphs]
    for d in datas:
        d.x = torch.round(d.x * 2)
        d.cluster1 = torch.tensor([i % 2 for i in range(len(d.cluster1))])
    torch.manual_seed(0)
    model = gnn_ref.GINet(30, 1, 3)
    for p in model.parameters():
        p.data = torch.round(p.data * 8) / 8
    model.eval()
    bat = P.Batch.from_data_list(datas)
    out = model(bat.clone())
    loss = torch.nn.functional.mse_loss(out.reshape(-1), bat.y)
    loss.backward()
    recs = records_from_batch(P.Batch.from_data_list(datas))
    params = [dict(model.named_parameters())[n].detach().numpy() for n in PARAM_NAMES]
    mout, grads, _ = M.run(pack_graphs(recs), params, 1, loss="mse")
    np.testing.assert_allclose(mout, out.detach().numpy(), rtol=1e-5, atol=1e-5)
    for i, n in enumerate(PARAM_NAMES):
        np.testing.assert_allclose(grads[i], dict(model.named_parameters())[n].grad.numpy(), rtol=1e-4, atol=1e-5, err_msg=n)


def _random_records(seed, n_graphs=12, asym=True):
    from deeprank2_amd.store import GraphRecord

    rng = np.random.default_rng(seed)
    recs = []
    for g in range(n_graphs):
        n = int(rng.integers(1, 40))
        e = int(rng.integers(0, 4 * n))
        ei = rng.integers(0, n, size=(2, e))
        if not asym:
            ei = np.concatenate([ei, ei[::-1]], 1)
        if g % 3 == 0 and n > 2:  # duplicates and self loops
            ei = np.concatenate([ei, np.array([[0, 0, 1], [0, 1, 1]])], 1)
        k = int(rng.integers(1, min(n, 6) + 1))
        c0 = rng.integers(0, k, size=n) * (3 if g % 2 else 1)  # non-consecutive ids
        k0 = len(np.unique(c0))
        c1 = rng.integers(0, 2, size=k0)
        recs.append(GraphRecord(x=rng.normal(size=(n, 7)).astype(np.float32), edge_index=ei, edge_attr=rng.normal(size=(ei.shape[1], 2)).astype(np.float32), cluster0=c0, cluster1=c1, y=float(g), name=f"r{g}"))
    return recs


@pytest.mark.parametrize("asym", [True, False])
def test_native_packer_matches_numpy_model(asym):
    from pack_model import pack_graphs_numpy

    recs = _random_records(11 + asym, asym=asym)
    a, b = pack_graphs(recs), pack_graphs_numpy(recs)
    for f in ("node_off", "edge_off", "rowptr", "col", "eperm", "t_rowptr", "t_col", "t_eid", "k0_off", "m0_ptr", "m0_idx", "cl0", "p1_off", "p1_rowptr", "p1_col", "p1t_rowptr", "p1t_col", "p1t_pid", "k1_off", "m1_ptr", "m1_idx", "cl1", "edge_attr", "p1_ea", "x", "y"):
        np.testing.assert_array_equal(getattr(a, f), getattr(b, f), err_msg=f)
    assert a.transpose_aliased == b.transpose_aliased


def test_native_packer_errors_and_missing_clusters():
    recs = _random_records(3, n_graphs=4)
    recs[2].cluster1 = np.array([0])
    recs[2].cluster0 = np.array([0, 5] * 50)[: len(recs[2].x)]
    if len(np.unique(recs[2].cluster0)) != 1:
        with pytest.raises(ValueError, match="cluster1"):
            pack_graphs(recs)
    recs = _random_records(4, n_graphs=3)
    recs[1].edge_index = np.array([[0], [999]])
    recs[1].edge_attr = np.zeros((1, 2), np.float32)
    with pytest.raises(ValueError, match="out of range"):
        pack_graphs(recs)
    recs = _random_records(5, n_graphs=3)
    for r in recs:
        r.cluster0 = r.cluster1 = None
    with pytest.raises(ValueError, match="cluster0/cluster1"):
        pack_graphs(recs)
    p = pack_graphs(recs, require_clusters=False)
    assert not p.has_clusters and p.m1_ptr.tolist() == [0, 1] * 3


def test_nonfinite_flag_per_graph(golden):
    """The packer flags each graph holding a non-finite x / edge_attr entry
    (GINet routes those batches to the layer path that computes the attention)."""
    from _util import golden_batch

    from deeprank2_amd.store import nonfinite_graphs

    z = golden("ginet_nonfinite_all")
    p = pack_graphs(records_from_batch(golden_batch(z)))
    assert p.nonfinite.tolist() == [True, True, True, False, False]
    x = np.zeros((6, 2), np.float32)
    x[4, 1] = np.inf
    ea = np.zeros((5, 1), np.float32)
    ea[0, 0] = np.nan
    assert nonfinite_graphs(x, np.array([0, 2, 4, 6]), ea, np.array([0, 1, 3, 5])).tolist() == [True, False, True]
    assert nonfinite_graphs(x[:0], np.array([0])).tolist() == []
