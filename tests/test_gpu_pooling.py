"""Layer-level pooling helpers on the GPU (dr_segment_max / _bwd / mean) against
the reference golden (community_pooling on 1ATN) and the oracle's
torch_scatter / PyG restatements (NaN and tie semantics, gradients)."""

from __future__ import annotations

import numpy as np
import pytest
import torch
from _util import golden_batch

from deeprank2_amd.data import Batch
from deeprank2_amd.utils import community_pooling as CP
from oracle import pyg_ops as P

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


def _gpu_batch(b):
    return Batch(**{k: (v.to(DEV) if isinstance(v, torch.Tensor) else v) for k, v in b.__dict__.items()})


def test_community_pooling_matches_golden(golden):
    z = golden("community_pooling_1atn")
    b = golden_batch(z)
    c = CP.get_preloaded_cluster(b.cluster0.clone().to(DEV), b.batch.to(DEV))
    np.testing.assert_array_equal(c.cpu().numpy(), z["out/cluster_offset"])
    pooled = CP.community_pooling(c, _gpu_batch(b))
    np.testing.assert_array_equal(pooled.x.cpu().numpy(), z["out/x"])
    np.testing.assert_array_equal(pooled.edge_index.cpu().numpy(), z["out/edge_index"])
    np.testing.assert_allclose(pooled.edge_attr.cpu().numpy(), z["out/edge_attr"], rtol=1e-6)
    np.testing.assert_array_equal(pooled.batch.cpu().numpy(), z["out/batch"])
    np.testing.assert_allclose(pooled.pos.cpu().numpy(), z["out/pos"], rtol=1e-5, atol=1e-5)


def _with_nan_and_ties():
    g = torch.Generator().manual_seed(3)
    x = torch.round(torch.randn(60, 7, generator=g) * 2) / 2  # ties
    x[4, 2] = float("nan")
    x[17, :] = float("nan")
    cluster = torch.randint(0, 9, (60,), generator=g) * 3  # non-consecutive ids
    return x, cluster


def test_scatter_max_semantics_and_grad_vs_oracle():
    x, cluster = _with_nan_and_ties()
    dense, _ = CP.consecutive_cluster(cluster)
    k = int(dense.max()) + 1
    xo = x.clone().requires_grad_(True)
    out_o, arg_o = P.scatter_max(xo, dense, dim=0)
    xa = x.to(DEV).requires_grad_(True)
    out_a, arg_a = CP.segment_max(xa, dense.to(DEV), k, CP.SCATTER_MAX)
    np.testing.assert_array_equal(out_a.detach().cpu().numpy(), out_o.detach().numpy())
    np.testing.assert_array_equal(arg_a.cpu().numpy(), arg_o.numpy())
    w = torch.randn(out_o.shape, generator=torch.Generator().manual_seed(1))
    (out_o * w).sum().backward()
    (out_a * w.to(DEV)).sum().backward()
    np.testing.assert_array_equal(xa.grad.cpu().numpy(), xo.grad.numpy())


def test_max_pool_x_amax_nan_and_ties_vs_oracle():
    x, cluster = _with_nan_and_ties()
    batch = torch.zeros(60, dtype=torch.long)
    xo = x.clone().requires_grad_(True)
    out_o, b_o = P.max_pool_x(cluster, xo, batch)
    xa = x.to(DEV).requires_grad_(True)
    out_a, b_a = CP.max_pool_x(cluster.to(DEV), xa, batch.to(DEV))
    np.testing.assert_array_equal(out_a.detach().cpu().numpy(), out_o.detach().numpy())
    np.testing.assert_array_equal(b_a.cpu().numpy(), b_o.numpy())
    w = torch.randn(out_o.shape, generator=torch.Generator().manual_seed(2))
    (out_o * w).sum().backward()
    (out_a * w.to(DEV)).sum().backward()
    np.testing.assert_allclose(xa.grad.cpu().numpy(), xo.grad.numpy(), rtol=1e-6, equal_nan=True)
