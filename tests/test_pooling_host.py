"""Integer side of the pooling helpers on CPU (tensor ops, no kernels):
get_preloaded_cluster / consecutive_cluster / pool_edge against the
community_pooling golden of the reference on 1ATN."""

from __future__ import annotations

import numpy as np
import torch
from _util import golden_batch

from deeprank2_amd.utils import community_pooling as CP


def test_cluster_offsets_and_pooled_edges_match_golden(golden):
    z = golden("community_pooling_1atn")
    b = golden_batch(z)
    c = CP.get_preloaded_cluster(b.cluster0.clone(), b.batch)
    np.testing.assert_array_equal(c.numpy(), z["out/cluster_offset"])
    dense, perm = CP.consecutive_cluster(c)
    ei, ea = CP.pool_edge(dense, b.edge_index, b.edge_attr)
    np.testing.assert_array_equal(ei.numpy(), z["out/edge_index"])
    np.testing.assert_allclose(ea.numpy(), z["out/edge_attr"], rtol=1e-6)
    np.testing.assert_array_equal(b.batch[perm].numpy(), z["out/batch"])


def test_get_preloaded_cluster_is_in_place():
    c = torch.tensor([0, 1, 1, 0, 2, 0, 0])
    batch = torch.tensor([0, 0, 0, 1, 1, 2, 2])
    out = CP.get_preloaded_cluster(c, batch)
    assert out is c
    assert c.tolist() == [0, 1, 1, 2, 4, 5, 5]
