"""MCL community detection (Trainer._precluster, trainer.py:319-348;
community_pooling.py:96-162): the oracle pinned by the clusters the reference
stored, and the host-side layout / pooling / assignment logic."""

from __future__ import annotations

import glob
import os

import numpy as np
import pytest
import torch
from _util import golden_graphs

from deeprank2_amd import clustering
from deeprank2_amd.utils import community_pooling as CP
from oracle import mcl_ref
from oracle import pyg_ops as P

REF_H5 = "/root/reference/tests/data/hdf5"


@pytest.mark.parametrize("name", ["ginet_1atn", "foutnet_testhdf5"])
def test_oracle_reproduces_stored_depth0_depth1(golden, name):
    """depth_0 on the graph, depth_1 on the pooled graph == the stored clusters."""
    for ei, n, c0, c1 in golden_graphs(golden(name)):
        a = mcl_ref.mcl_community_detection(ei, n)
        np.testing.assert_array_equal(a, c0)
        pe, k = clustering.pooled_graph(a, ei)
        np.testing.assert_array_equal(mcl_ref.mcl_community_detection(pe, k), c1)


@pytest.mark.skipif(not os.path.isdir(REF_H5), reason="reference fixtures not present")
def test_oracle_reproduces_reference_hdf5_clusters():
    """Every entry of the reference's fixtures that stores clustering/mcl."""
    from deeprank2_amd.io import hdf5  # noqa: PLC0415

    files = sorted(glob.glob(f"{REF_H5}/*.hdf5"))
    seen = 0
    for p, d in zip(files, hdf5.read_files(files)):
        if isinstance(d, Exception):
            continue
        for entry, g in d.items():
            if "clustering/mcl/depth_0" not in g:
                continue
            ind = g["edge_features/_index"]
            ei = np.vstack((ind, np.flip(ind, 1))).T
            n = g["node_features/_position"].shape[0]
            a = mcl_ref.mcl_community_detection(ei, n)
            np.testing.assert_array_equal(a, g["clustering/mcl/depth_0"], err_msg=f"{p}:{entry}")
            pe, k = clustering.pooled_graph(a, ei)
            np.testing.assert_array_equal(mcl_ref.mcl_community_detection(pe, k), g["clustering/mcl/depth_1"], err_msg=f"{p}:{entry}")
            seen += 1
    assert seen >= 10


def test_pooled_graph_matches_pool_edge():
    rng = np.random.default_rng(3)
    for _ in range(5):
        n = int(rng.integers(5, 40))
        ei = rng.integers(0, n, size=(2, 4 * n))
        c = rng.integers(0, 7, size=n) * 3  # non-consecutive ids
        pe, k = clustering.pooled_graph(c, ei)
        dense, perm = P.consecutive_cluster(torch.from_numpy(c))
        ref, _ = P.pool_edge(dense, torch.from_numpy(ei), None)
        assert k == perm.numel()
        np.testing.assert_array_equal(pe, ref.numpy())


def test_layout_is_local_csr_per_graph():
    rng = np.random.default_rng(5)
    graphs = []
    for n in (1, 0, 17, 64, 65, 130):
        e = int(rng.integers(0, 5 * n + 1)) if n else 0
        graphs.append((rng.integers(0, max(n, 1), size=(2, e)), n))
    n, node_off, rowptr, edge_off, col, w = clustering._layout(graphs, None)  # noqa: SLF001
    assert w is None and rowptr.size == node_off[-1] + len(graphs)
    for g, (ei, nn) in enumerate(graphs):
        rp = rowptr[node_off[g] + g : node_off[g] + g + nn + 1]
        assert rp[0] == 0 and rp[-1] == ei.shape[1] == edge_off[g + 1] - edge_off[g]
        got = sorted((i, int(col[edge_off[g] + e])) for i in range(nn) for e in range(rp[i], rp[i + 1]))
        assert got == sorted(zip(ei[0].tolist(), ei[1].tolist()))


def test_layout_rejects_out_of_range_edges():
    with pytest.raises(ValueError, match="outside"):
        clustering._layout([(np.array([[0], [5]]), 3)], None)  # noqa: SLF001


def test_weighted_edges_last_weight_wins_symmetrically():
    s, d, w = clustering._symmetric_weighted(np.array([0, 1, 2, 0]), np.array([1, 0, 0, 2]), np.array([1.0, 2.0, 3.0, 4.0]))  # noqa: SLF001
    got = {(int(a), int(b)): float(c) for a, b, c in zip(s, d, w)}
    assert got == {(0, 1): 2.0, (1, 0): 2.0, (0, 2): 4.0, (2, 0): 4.0}


def test_oracle_adjacency_matches_networkx_semantics():
    ei = np.array([[0, 1, 1, 2, 2], [1, 0, 2, 1, 2]])
    assert mcl_ref.adjacency(ei, 4).tolist() == [[0, 1, 0, 0], [1, 0, 1, 0], [0, 1, 1, 0], [0, 0, 0, 0]]
    w = mcl_ref.adjacency(ei, 3, np.array([5.0, 6.0, 7.0, 8.0, 9.0]))
    assert w.tolist() == [[0, 6, 0], [6, 0, 8], [0, 8, 9]]


def test_community_detection_method_checks():
    ei = torch.tensor([[0, 1], [1, 0]])
    with pytest.raises(NotImplementedError):
        CP.community_detection(ei, 2, method="louvain")
    with pytest.raises(ValueError, match="not supported"):
        CP.community_detection(ei, 2, method="kmeans")
    if not torch.cuda.is_available():
        with pytest.raises(RuntimeError, match="no CPU fallback"):
            CP.community_detection(ei, 2)
        with pytest.raises(RuntimeError, match="no CPU fallback"):
            clustering.mcl_clusters([(ei.numpy(), 2)], "cpu")
