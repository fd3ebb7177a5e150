"""Layer-level execution of FoutNet, SGAT and ``ginet_nocluster.GINet`` for
batches their per-graph kernels cannot hold (a graph beyond one workgroup's
160 KiB of LDS, e.g. atom-level graphs).  GINet and VanillaNetwork have
split large-graph kernels of their own for that.  GINet and
``ginet_nocluster.GINet`` also come here for batches holding a non-finite
``x`` / ``edge_attr`` entry: their kernels take the attention as identically 1,
which holds only for finite logits (ginet.py:48-54).

The forward mirrors the reference line by line on the layer API — FoutLayer /
SGraphAttentionLayer / GINetConvLayer on the CSR and linear HIP kernels,
``get_preloaded_cluster`` / ``community_pooling`` / ``max_pool_x`` on the
segment kernels (``deeprank2_amd.utils.community_pooling``), ``nn.Linear`` on
rocBLAS — and torch autograd differentiates it:
  * FoutNet.forward          deeprank2/neuralnets/gnn/foutnet.py:99-118
  * SGAT.forward             deeprank2/neuralnets/gnn/sgat.py:113-133
  * ginet_nocluster.GINet    deeprank2/neuralnets/gnn/ginet_nocluster.py:84-111
  * GINet.forward            deeprank2/neuralnets/gnn/ginet.py:90-125
The batch tensors come from the HBM store the batch handle points into
(``batch_tensors``), in the reference's edge order (the store's CSR slot map
``eperm``), so each scatter sums in the same order as the reference.
"""

from __future__ import annotations

from types import SimpleNamespace

import numpy as np
import torch
from torch.nn.functional import dropout, relu

from deeprank2_amd.fused import LDS_MAX, BatchHandle, FusedSpec, lds_for
from deeprank2_amd.utils.community_pooling import AMAX, SCATTER_MAX, _segments, _SegmentMax, consecutive_cluster, get_preloaded_cluster, pool_edge


def needs_layers(spec: FusedSpec, h: BatchHandle, out_dim) -> bool:
    """True when ``spec``'s graph pass cannot run this batch: no split
    large-graph path and the largest graph exceeds one workgroup's LDS (or the
    handle asks for the layer path: ``h.force_layers``, a diagnostic)."""
    if getattr(h, "force_layers", False):
        return True
    if spec.layers is None:
        return False
    if spec.attention and getattr(h, "nonfinite", False):
        return True
    if spec.run is not None or spec.large is not None:
        return False
    return lds_for(spec, h, out_dim) > LDS_MAX


def batch_tensors(h: BatchHandle):
    """The batch as the reference's collated ``Batch`` holds it (x, edge_index
    in the original edge order, edge_attr, batch vector, cluster0 / cluster1 as
    dense per-graph ids, y), on the store's device; built once per handle."""
    t = h._lds.get("layer_tensors")  # noqa: SLF001
    if t is not None:
        return t
    p = h.store.packed
    xs, eis, eas, bs, c0s, c1s = [], [], [], [], [], []
    base = 0
    for slot, gid in enumerate(h.gids_host.astype(np.int64)):
        n0, n1 = int(p.node_off[gid]), int(p.node_off[gid + 1])
        e0, e1 = int(p.edge_off[gid]), int(p.edge_off[gid + 1])
        n, e = n1 - n0, e1 - e0
        rp = p.rowptr[n0 + gid : n1 + gid + 1].astype(np.int64)
        rows = np.repeat(np.arange(n, dtype=np.int64), np.diff(rp))
        cols = p.col[e0:e1].astype(np.int64)
        pos = p.eperm[e0:e1].astype(np.int64)  # CSR slot -> original edge position
        ei = np.empty((2, e), np.int64)
        ei[0, pos], ei[1, pos] = rows, cols
        eis.append(ei + base)
        if p.edge_attr is not None:
            ea = np.empty_like(p.edge_attr[e0:e1])
            ea[pos] = p.edge_attr[e0:e1]
            eas.append(ea)
        xs.append(p.x[n0:n1])
        bs.append(np.full(n, slot, np.int64))
        c0s.append(p.cl0[n0:n1].astype(np.int64))
        c1s.append(p.cl1[int(p.k0_off[gid]) : int(p.k0_off[gid + 1])].astype(np.int64))
        base += n
    dev = h.store.device
    d = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(dev)  # noqa: E731
    t = SimpleNamespace(
        x=d(np.concatenate(xs)),
        edge_index=d(np.concatenate(eis, axis=1)),
        edge_attr=d(np.concatenate(eas)) if eas else None,
        batch=d(np.concatenate(bs)),
        cluster0=d(np.concatenate(c0s)),
        cluster1=d(np.concatenate(c1s)),
        y=d(p.y[h.gids_host.astype(np.int64)]),
        n_graphs=h.B,
    )
    h._lds["layer_tensors"] = t  # noqa: SLF001
    return t


def scatter_mean(x, batch, n_seg):
    """torch_scatter.scatter_mean over graphs (count clamped at 1), differentiable."""
    s = torch.zeros(n_seg, x.shape[1], dtype=x.dtype, device=x.device).index_add(0, batch, x)
    cnt = torch.zeros(n_seg, dtype=x.dtype, device=x.device).index_add(0, batch, torch.ones_like(batch, dtype=x.dtype))
    return s / cnt.clamp_min(1).unsqueeze(1)


def pool_plan(t):
    """The batch-static part of ``community_pooling`` and ``max_pool_x``
    (community_pooling.py:23-27,165-242; PyG consecutive_cluster / pool_edge /
    pool_batch): offset and relabelled clusters of both depths with their
    segment lists, the pooled graph (coalesced edge_attr sums) and the pooled
    batch vectors — a pure function of the batch's graphs, built once per
    batch (cached on the batch tensors) instead of once per forward (each
    build syncs with the host).  Only the feature max-pools run per step."""
    pl = getattr(t, "pool_plan", None)
    if pl is None:
        dense0, perm0 = consecutive_cluster(get_preloaded_cluster(t.cluster0.clone(), t.batch))
        k0 = int(perm0.numel())
        ei1, ea1 = pool_edge(dense0, t.edge_index, t.edge_attr)
        batch1 = t.batch[perm0]
        dense1, perm1 = consecutive_cluster(get_preloaded_cluster(t.cluster1.clone(), batch1))
        k1 = int(perm1.numel())
        pl = SimpleNamespace(k0=k0, seg0=_segments(dense0, k0), ei1=ei1, ea1=ea1, k1=k1, seg1=_segments(dense1, k1), batch2=batch1[perm1])
        t.pool_plan = pl
    return pl


def _pool0(pl, x):
    """scatter_max of community_pooling (torch_scatter: NaN dropped, first max)."""
    return _SegmentMax.apply(x, pl.seg0[0], pl.seg0[1], pl.k0, SCATTER_MAX)[0]


def _pooled_head(model, t, x1, with_edge_attr):
    """conv2 block, depth-1 max_pool_x, per-graph mean and the MLP head
    (foutnet.py:107-118, sgat.py:123-133)."""
    pl = pool_plan(t)
    if with_edge_attr:
        x = relu(model.conv2(x1, pl.ei1, pl.ea1))
    else:
        x = relu(model.conv2(x1, pl.ei1))
    x = _SegmentMax.apply(x, pl.seg1[0], pl.seg1[1], pl.k1, AMAX)[0]  # max_pool_x (amax: NaN propagates)
    x = scatter_mean(x, pl.batch2, t.n_graphs)
    x = relu(model.fc1(x))
    return model.fc2(x)


def _dropout(model, g, training, mask):
    """Dropout of the head (ginet.py:122): the explicit uint8 keep mask
    [B, 128] if given (tests, as the fused kernels take it), else torch's RNG."""
    if not training or model.dropout <= 0:
        return g
    if mask is not None:
        return g * mask.to(device=g.device, dtype=g.dtype) * (1.0 / (1.0 - model.dropout))
    return dropout(g, model.dropout, training=True)


def ginet_forward(model, t, training=False, mask=None):
    """ginet.py:90-125, both branches, with GINetConvLayer's attention computed
    whenever its inputs are non-finite (``ginet._attention_conv``)."""
    pl = pool_plan(t)

    def branch(conv_a, conv_b):
        x = _pool0(pl, relu(conv_a(t.x, t.edge_index, t.edge_attr)))
        x = relu(conv_b(x, pl.ei1, pl.ea1))
        x = _SegmentMax.apply(x, pl.seg1[0], pl.seg1[1], pl.k1, AMAX)[0]
        return scatter_mean(x, pl.batch2, t.n_graphs)

    g = torch.cat([branch(model.conv1, model.conv2), branch(model.conv1_ext, model.conv2_ext)], dim=1)
    g = _dropout(model, relu(model.fc1(g)), training, mask)
    return model.fc2(g)


def foutnet_forward(model, t, training=False, mask=None):  # noqa: ARG001
    """foutnet.py:99-118."""
    x = _pool0(pool_plan(t), relu(model.conv1(t.x, t.edge_index)))
    return _pooled_head(model, t, x, with_edge_attr=False)


def sgat_forward(model, t, training=False, mask=None):  # noqa: ARG001
    """sgat.py:113-133 (pooled edge_attr = PyG coalesce sums, as community_pooling gives)."""
    x = _pool0(pool_plan(t), relu(model.conv1(t.x, t.edge_index, t.edge_attr)))
    return _pooled_head(model, t, x, with_edge_attr=True)


def ginet_nocluster_forward(model, t, training=False, mask=None):
    """ginet_nocluster.py:84-111 (dropout: the keep mask if given, else torch's RNG)."""
    ea = t.edge_attr
    x = relu(model.conv1(t.x, t.edge_index, ea))
    x = relu(model.conv2(x, t.edge_index, ea))
    x_ext = relu(model.conv1_ext(t.x, t.edge_index, ea))
    x_ext = relu(model.conv2_ext(x_ext, t.edge_index, ea))
    g = torch.cat([scatter_mean(x, t.batch, t.n_graphs), scatter_mean(x_ext, t.batch, t.n_graphs)], dim=1)
    g = _dropout(model, relu(model.fc1(g)), training, mask)
    return model.fc2(g)
