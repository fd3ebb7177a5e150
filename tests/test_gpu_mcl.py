"""dr_mcl (fp64 MCL on the GPU) + dr_mcl_assign against the oracle
(oracle/mcl_ref.py, pinned by the reference's stored clusters) and the stored
clusters themselves; Trainer._precluster end to end."""

from __future__ import annotations

import numpy as np
import pytest
import torch
from _util import golden_graphs

from deeprank2_amd import clustering
from deeprank2_amd.utils import community_pooling as CP
from deeprank2_amd.utils import synthetic as S
from oracle import mcl_ref

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["ginet_1atn", "foutnet_testhdf5"])
def test_gpu_reproduces_stored_clusters(golden, name):
    gs = golden_graphs(golden(name))
    c0, c1 = clustering.precluster_graphs([(ei, n) for ei, n, _, _ in gs], "cuda:0")
    for (_, _, r0, r1), a, b in zip(gs, c0, c1):
        np.testing.assert_array_equal(a, r0)
        np.testing.assert_array_equal(b, r1)


def _synthetic(seed, count):
    rng = np.random.default_rng(seed)
    out = [(np.zeros((2, 0), np.int64), 0), (np.zeros((2, 0), np.int64), 1), (np.array([[0, 1], [1, 0]]), 5)]  # empty, single, isolated nodes
    for g in S.make_dataset(count, seed=seed, n_lo=20, n_hi=300, mean_degree=6.0):
        out.append((g["index"].T.copy(), g["x"].shape[0]))
    for n in (63, 64, 65, 129):  # tile edges of the 64-wide expansion
        e = rng.integers(0, n, size=(2, 3 * n))
        out.append((e, n))
    return out


def test_gpu_matches_oracle_on_varied_graphs():
    graphs = _synthetic(21, 24)
    got, iters = clustering.mcl_clusters(graphs, "cuda:0", return_iters=True)
    for (ei, n), a, it in zip(graphs, got, iters):
        if n == 0:  # markov_clustering raises on an empty matrix; here: no nodes, no ids
            assert a.size == 0
            continue
        ref = mcl_ref.mcl_community_detection(ei, n)
        np.testing.assert_array_equal(a, ref, err_msg=f"n={n}")
        assert 1 <= it <= clustering.MAX_ITER or n == 0


def test_gpu_chunked_launches_match(monkeypatch):
    graphs = _synthetic(22, 10)
    whole = clustering.mcl_clusters(graphs, "cuda:0")
    monkeypatch.setattr(clustering, "WORKSPACE_BUDGET", 1 << 20)  # forces several launches
    for a, b in zip(whole, clustering.mcl_clusters(graphs, "cuda:0")):
        np.testing.assert_array_equal(a, b)


def test_gpu_weighted_community_detection():
    rng = np.random.default_rng(4)
    for n in (12, 40, 90):
        ei = rng.integers(0, n, size=(2, 4 * n))
        w = rng.uniform(0.1, 3.0, size=ei.shape[1])
        got = CP.community_detection(torch.from_numpy(ei).cuda(), n, edge_attr=torch.from_numpy(w))
        assert got.is_cuda and got.dtype == torch.int64
        np.testing.assert_array_equal(got.cpu().numpy(), mcl_ref.mcl_community_detection(ei, n, w))


def test_trainer_precluster_installs_mcl_clusters(tmp_path):
    from deeprank2_amd.dataset import GraphDataset  # noqa: PLC0415
    from deeprank2_amd.neuralnets.gnn.ginet import GINet  # noqa: PLC0415
    from deeprank2_amd.trainer import Trainer  # noqa: PLC0415

    tr_p, va_p = str(tmp_path / "tr.hdf5"), str(tmp_path / "va.hdf5")
    S.write_hdf5(tr_p, S.make_dataset(6, seed=31, n_lo=25, n_hi=60), prefix="tr")
    S.write_hdf5(va_p, S.make_dataset(3, seed=32, n_lo=25, n_hi=60), prefix="va")
    tr = GraphDataset(tr_p, node_features=S.SYNTH_NODE_FEATURES, edge_features=S.SYNTH_EDGE_FEATURES, target="irmsd", clustering_method="mcl")
    va = GraphDataset(va_p, train_source=tr, clustering_method="mcl")
    t = Trainer(GINet, tr, va, cuda=True)
    for ds in (t.dataset_train, t.dataset_val):
        for i in range(len(ds)):
            d = ds.get(i)
            ei = d.edge_index.numpy()
            c0 = mcl_ref.mcl_community_detection(ei, d.num_nodes)
            np.testing.assert_array_equal(d.cluster0.numpy(), c0)
            pe, k = clustering.pooled_graph(c0, ei)
            np.testing.assert_array_equal(d.cluster1.numpy(), mcl_ref.mcl_community_detection(pe, k))
    t.train(nepoch=1, batch_size=4, validate=True, best_model=False, filename=None)
