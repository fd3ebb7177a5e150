"""Cluster pooling helpers — drop-in for ``deeprank2.utils.community_pooling``
(``get_preloaded_cluster``, ``community_pooling``) plus PyG's ``max_pool_x``
as the reference networks call it.

The fused models never call these (their pooling is precomputed into the
graph store and done inside the kernels); they are the layer-level API for
code that builds its own networks.  Feature pooling runs on the HIP segment
kernels (``dr_segment_max`` with the torch_scatter / amax semantics, and its
backward; ``dr_segment_mean``); cluster relabelling and edge coalescing are
integer bookkeeping done with device tensor ops.
Reference: ``deeprank2/utils/community_pooling.py:23-27,165-242``; PyG 2.4
``consecutive_cluster`` / ``pool_edge`` / ``pool_batch`` / ``max_pool_x``.
``community_detection(method="mcl")`` runs the batched fp64 MCL kernel
(``deeprank2_amd.clustering``); Louvain (randomised ``python-louvain``) is not
provided.
"""

from __future__ import annotations

import warnings

import torch

from deeprank2_amd import _lib, ops
from deeprank2_amd.data import Batch, Data

SCATTER_MAX, AMAX = 0, 1


def get_preloaded_cluster(cluster, batch):
    """community_pooling.py:23-27: offset each graph's cluster ids past the
    previous graph's (in place, like the reference)."""
    nb = int(batch.max()) + 1 if batch.numel() else 0
    if nb <= 1:
        return cluster
    mx = torch.full((nb,), torch.iinfo(cluster.dtype).min, dtype=cluster.dtype, device=cluster.device)
    mx.scatter_reduce_(0, batch, cluster, "amax")
    off = torch.zeros(nb, dtype=cluster.dtype, device=cluster.device)
    off[1:] = torch.cumsum(mx[:-1] + 1, 0)  # offset_b = offset_{b-1} + max_{b-1} + 1 (raw ids)
    cluster += off[batch]
    return cluster


def consecutive_cluster(src):
    """PyG consecutive_cluster: dense ids (sorted unique) and one member per cluster."""
    uniq, inv = torch.unique(src, sorted=True, return_inverse=True)
    perm = torch.empty(uniq.numel(), dtype=torch.long, device=src.device)
    perm.scatter_(0, inv, torch.arange(inv.numel(), device=src.device))
    return inv, perm


def _segments(dense, n_seg):
    segptr, _, members = ops.csr_from_coo(dense, torch.arange(dense.numel(), device=dense.device), n_seg)
    return segptr, members


class _SegmentMax(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, segptr, members, n_seg, mode):
        x = x.contiguous().float()
        n, c = x.shape
        out = torch.empty(n_seg, c, dtype=torch.float32, device=x.device)
        arg = torch.empty(n_seg, c, dtype=torch.int32, device=x.device)
        _lib.check(_lib.load().dr_segment_max(segptr.data_ptr(), members.data_ptr(), x.data_ptr(), n_seg, c, n, mode, out.data_ptr(), arg.data_ptr(), _lib.stream_ptr(x.device)), "dr_segment_max")
        ctx.save_for_backward(x, segptr, members, out, arg)
        ctx.mode, ctx.n_seg = mode, n_seg
        ctx.mark_non_differentiable(arg)
        return out, arg

    @staticmethod
    def backward(ctx, dout, _darg):
        x, segptr, members, out, arg = ctx.saved_tensors
        n, c = x.shape
        dx = torch.zeros_like(x)
        _lib.check(_lib.load().dr_segment_max_bwd(segptr.data_ptr(), members.data_ptr(), x.data_ptr(), out.data_ptr(), arg.data_ptr(), dout.contiguous().data_ptr(), ctx.n_seg, c, n, ctx.mode, dx.data_ptr(), _lib.stream_ptr(x.device)), "dr_segment_max_bwd")
        return dx, None, None, None, None


def segment_max(x, dense, n_seg, mode=SCATTER_MAX):
    """(out [n_seg, C], arg [n_seg, C]) of a dense cluster vector."""
    _lib.require_device(x, dense)
    segptr, members = _segments(dense, n_seg)
    return _SegmentMax.apply(x, segptr, members, n_seg, mode)


def segment_mean(x, dense, n_seg):
    _lib.require_device(x, dense)
    x = x.contiguous().float()
    segptr, members = _segments(dense, n_seg)
    out = torch.empty(n_seg, x.shape[1], dtype=torch.float32, device=x.device)
    _lib.check(_lib.load().dr_segment_mean(segptr.data_ptr(), members.data_ptr(), x.data_ptr(), n_seg, x.shape[1], out.data_ptr(), _lib.stream_ptr(x.device)), "dr_segment_mean")
    return out


def community_detection(edge_index, num_nodes: int, edge_attr=None, method: str = "mcl"):
    """community_pooling.py:96-162: cluster id per node (int64, on
    ``edge_index``'s device).  MCL runs on the GPU (``dr_mcl``) with
    markov_clustering's defaults; ``edge_attr`` (one weight per edge) gives the
    weighted adjacency networkx builds (last weight of a repeated pair wins)."""
    if method == "louvain":
        msg = "Louvain clustering (python-louvain best_partition, randomised) is not provided by deeprank2_amd; use method='mcl'"
        raise NotImplementedError(msg)
    if method != "mcl":
        msg = f"Clustering method {method} not supported"
        raise ValueError(msg)
    from deeprank2_amd import clustering  # noqa: PLC0415

    dev = edge_index.device if edge_index.is_cuda else None
    if dev is None and not torch.cuda.is_available():
        msg = "community_detection runs on the MI355X only (no CPU fallback by design)"
        raise RuntimeError(msg)
    ei = edge_index.detach().cpu().numpy()
    w = None if edge_attr is None else [torch.as_tensor(edge_attr).detach().cpu().double().reshape(-1).numpy()]
    (c,) = clustering.mcl_clusters([(ei, int(num_nodes))], dev, weights=w)
    return torch.from_numpy(c).to(edge_index.device)


def pool_edge(cluster, edge_index, edge_attr=None):
    """PyG pool_edge: relabel, drop self loops, coalesce (unique, sorted by
    (row, col); edge_attr summed)."""
    k = int(cluster.max()) + 1 if cluster.numel() else 0
    row, col = cluster[edge_index[0]], cluster[edge_index[1]]
    keep = row != col
    key = row[keep] * k + col[keep]
    uniq, inv = torch.unique(key, sorted=True, return_inverse=True)
    ei = torch.stack([uniq // k, uniq % k]) if k else edge_index[:, :0]
    ea = None
    if edge_attr is not None:
        src = edge_attr[keep]
        ea = torch.zeros((uniq.numel(), *src.shape[1:]), dtype=src.dtype, device=src.device).index_add_(0, inv, src)
    return ei, ea


def community_pooling(cluster, data):
    """community_pooling.py:165-242: max-pool features (torch_scatter
    scatter_max), pool edges, mean-pool positions, pool the batch vector."""
    if hasattr(data, "internal_edge_index") and getattr(data, "internal_edge_index", None) is not None:
        warnings.warn("Internal edges are not supported anymore. Please prepare the hdf5 file with a more up to date version of this software.", DeprecationWarning, stacklevel=2)
    dense, perm = consecutive_cluster(cluster)
    dense = dense.to(data.x.device)
    k = int(perm.numel())
    x, _ = segment_max(data.x, dense, k, SCATTER_MAX)
    edge_index, edge_attr = pool_edge(dense, data.edge_index, getattr(data, "edge_attr", None))
    pos = segment_mean(data.pos, dense, k) if getattr(data, "pos", None) is not None else None
    c0, c1 = getattr(data, "cluster0", None), getattr(data, "cluster1", None)
    bvec = getattr(data, "batch", None)
    if isinstance(data, Batch) or bvec is not None:
        out = Batch(batch=None if bvec is None else bvec[perm.to(bvec.device)], x=x, edge_index=edge_index, edge_attr=edge_attr, pos=pos)
    else:
        out = Data(x=x, edge_index=edge_index, edge_attr=edge_attr, pos=pos)
    out.cluster0, out.cluster1 = c0, c1
    return out


def max_pool_x(cluster, x, batch):
    """PyG max_pool_x (ginet.py:103, foutnet.py:111): amax per cluster (NaN
    propagates; ties share the gradient) and the pooled batch vector."""
    dense, perm = consecutive_cluster(cluster)
    out, _ = segment_max(x, dense.to(x.device), int(perm.numel()), AMAX)
    return out, batch[perm.to(batch.device)]
