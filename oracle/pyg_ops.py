"""TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

torch-CPU restatement of the third-party ops on the DeepRank2 GNN path.
Pins (``/root/reference/env/deeprank2_frozen.yml:77,81,84``): pyg 2.4.0,
pytorch 2.1.1, pytorch-scatter 2.1.2.  None of these packages is installed in
this image, so every function below restates the pinned version's documented
behaviour; parity at this boundary is UNPINNED.
"""

from __future__ import annotations

import copy
import math

import torch

# --------------------------------------------------------------------------
# torch_scatter 2.1.2  (call sites: ginet.py:58,117-118; foutnet.py:114;
# vanilla_gnn.py:35,62; community_pooling.py:209,216)
# --------------------------------------------------------------------------


def _broadcast(src: torch.Tensor, other: torch.Tensor, dim: int) -> torch.Tensor:
    if dim < 0:
        dim = other.dim() + dim
    if src.dim() == 1:
        for _ in range(dim):
            src = src.unsqueeze(0)
    for _ in range(src.dim(), other.dim()):
        src = src.unsqueeze(-1)
    return src.expand(other.size())


def scatter_sum(src, index, dim=0, out=None, dim_size=None):
    """``out.scatter_add_(dim, index, src)``; size ``index.max()+1`` when not given."""
    index = _broadcast(index, src, dim)
    if out is None:
        size = list(src.size())
        if dim_size is not None:
            size[dim] = dim_size
        elif index.numel() == 0:
            size[dim] = 0
        else:
            size[dim] = int(index.max()) + 1
        out = torch.zeros(size, dtype=src.dtype, device=src.device)
    return out.scatter_add_(dim, index, src)


def scatter_mean(src, index, dim=0, out=None, dim_size=None):
    """Segment sum divided by the member count clamped to >= 1."""
    out = scatter_sum(src, index, dim, out, dim_size)
    dim_size = out.size(dim)
    index_dim = dim if dim >= 0 else dim + src.dim()
    if index.dim() <= index_dim:
        index_dim = index.dim() - 1
    ones = torch.ones(index.size(), dtype=src.dtype, device=src.device)
    count = scatter_sum(ones, index, index_dim, None, dim_size)
    count[count < 1] = 1
    count = _broadcast(count, out, dim)
    if out.is_floating_point():
        out.true_divide_(count)
    else:
        out.div_(count, rounding_mode="floor")
    return out


class _ScatterMax(torch.autograd.Function):
    """torch_scatter CPU ``scatter_max`` along dim 0 for 2-D ``src``.

    Forward semantics (csrc/cpu/scatter_cpu.cpp + reducer.h): the output starts
    at ``lowest()``; members are visited in index order and replace the
    running value only when strictly greater (so NaN never enters, ties keep
    the first member); segments left at ``lowest()`` become 0 with arg = N.
    Backward: the gradient goes to the arg member only.
    """

    @staticmethod
    def forward(ctx, src, index, dim_size):
        n, c = src.shape
        lowest = torch.finfo(src.dtype).min
        valid = src > lowest  # False for NaN, -inf and lowest() itself
        idx2 = index.view(-1, 1).expand(n, c)
        vals = torch.where(valid, src, torch.full_like(src, -math.inf))
        out = torch.full((dim_size, c), -math.inf, dtype=src.dtype)
        out.scatter_reduce_(0, idx2, vals, reduce="amax", include_self=True)
        gathered = out.gather(0, idx2)
        cand = valid & (vals == gathered)
        pos = torch.arange(n).view(-1, 1).expand(n, c)
        pos = torch.where(cand, pos, torch.full_like(pos, n))
        arg = torch.full((dim_size, c), n, dtype=torch.long)
        arg.scatter_reduce_(0, idx2, pos, reduce="amin", include_self=True)
        out = torch.where(torch.isinf(out) & (out < 0), torch.zeros_like(out), out)
        ctx.save_for_backward(arg)
        ctx.n = n
        ctx.mark_non_differentiable(arg)
        return out, arg

    @staticmethod
    def backward(ctx, grad_out, grad_arg):  # noqa: ARG004
        (arg,) = ctx.saved_tensors
        n = ctx.n
        grad_src = grad_out.new_zeros((n + 1, grad_out.shape[1]))
        grad_src.scatter_(0, arg, grad_out)
        return grad_src[:n], None, None


def scatter_max(src, index, dim=0, out=None, dim_size=None):
    if dim != 0 or src.dim() != 2 or out is not None:  # noqa: PLR2004
        msg = "restatement covers dim=0, 2-D src, out=None (the only call shape on the path)"
        raise NotImplementedError(msg)
    if dim_size is None:
        dim_size = int(index.max()) + 1 if index.numel() > 0 else 0
    return _ScatterMax.apply(src, index, dim_size)


# --------------------------------------------------------------------------
# PyG 2.4.0 utilities
# --------------------------------------------------------------------------


def pyg_scatter(src, index, dim=0, dim_size=None, reduce="sum"):
    """``torch_geometric.utils.scatter`` on CPU (the reference's CI device).

    min/max on CPU go to ``new_zeros(size).scatter_reduce_(..., 'amax',
    include_self=False)``: NaN propagates, empty segments stay 0, and autograd
    splits the gradient evenly across tied members.
    """
    if dim_size is None:
        dim_size = int(index.max()) + 1 if index.numel() > 0 else 0
    size = list(src.size())
    size[dim] = dim_size
    if reduce in ("sum", "add"):
        return src.new_zeros(size).scatter_add_(dim, _broadcast(index, src, dim), src)
    if reduce == "mean":
        count = src.new_zeros(dim_size)
        count.scatter_add_(0, index, src.new_ones(src.size(dim)))
        count = count.clamp(min=1)
        out = src.new_zeros(size).scatter_add_(dim, _broadcast(index, src, dim), src)
        return out / _broadcast(count, out, dim)
    if reduce in ("min", "max"):
        return src.new_zeros(size).scatter_reduce_(dim, _broadcast(index, src, dim), src, reduce=f"a{reduce}", include_self=False)
    raise ValueError(reduce)


def consecutive_cluster(src):
    """``torch_geometric.nn.pool.consecutive.consecutive_cluster``."""
    unique, inv = torch.unique(src, sorted=True, return_inverse=True)
    perm = torch.arange(inv.size(0), dtype=inv.dtype, device=inv.device)
    perm = inv.new_empty(unique.size(0)).scatter_(0, inv, perm)
    return inv, perm


def remove_self_loops(edge_index, edge_attr=None):
    mask = edge_index[0] != edge_index[1]
    edge_index = edge_index[:, mask]
    if edge_attr is None:
        return edge_index, None
    return edge_index, edge_attr[mask]


def coalesce(edge_index, edge_attr=None, num_nodes=None, reduce="sum"):
    """``torch_geometric.utils.coalesce``: sort by (row, col), merge duplicates.

    Duplicate edge attributes are reduced with ``reduce`` ('sum' is the 2.4.0
    default, as recalled; unverifiable offline).
    """
    nnz = edge_index.size(1)
    if num_nodes is None:
        num_nodes = int(edge_index.max()) + 1 if nnz > 0 else 0
    idx = edge_index.new_empty(nnz + 1)
    idx[0] = -1
    idx[1:] = edge_index[0] * num_nodes + edge_index[1]
    idx[1:], perm = torch.sort(idx[1:])  # ascending; PyG uses index_sort
    edge_index = edge_index[:, perm]
    if edge_attr is not None:
        edge_attr = edge_attr[perm]
    mask = idx[1:] > idx[:-1]
    if bool(mask.all()):
        return edge_index, edge_attr
    edge_index = edge_index[:, mask]
    if edge_attr is None:
        return edge_index, None
    dim_size = edge_index.size(1)
    group = mask.cumsum(0) - 1
    edge_attr = pyg_scatter(edge_attr, group, 0, dim_size, reduce)
    return edge_index, edge_attr


def pool_edge(cluster, edge_index, edge_attr=None):
    """``torch_geometric.nn.pool.pool.pool_edge``."""
    num_nodes = cluster.size(0)
    edge_index = cluster[edge_index.view(-1)].view(2, -1)
    edge_index, edge_attr = remove_self_loops(edge_index, edge_attr)
    if edge_index.numel() > 0:
        edge_index, edge_attr = coalesce(edge_index, edge_attr, num_nodes)
    return edge_index, edge_attr


def pool_batch(perm, batch):
    return batch[perm]


def max_pool_x(cluster, x, batch, batch_size=None, size=None):  # noqa: ARG001
    """``torch_geometric.nn.pool.max_pool_x`` (size=None form used on the path)."""
    cluster, perm = consecutive_cluster(cluster)
    x = pyg_scatter(x, cluster, dim=0, dim_size=None, reduce="max")
    batch = pool_batch(perm, batch)
    return x, batch


def uniform(size, value):
    """``torch_geometric.nn.inits.uniform``: U(-1/sqrt(size), 1/sqrt(size))."""
    if value is None:
        return
    if isinstance(value, torch.Tensor):
        bound = 1.0 / math.sqrt(size)
        value.data.uniform_(-bound, bound)
    else:
        for v in value.parameters() if hasattr(value, "parameters") else []:
            uniform(size, v)


# --------------------------------------------------------------------------
# PyG Data / Batch (only what the path touches)
# --------------------------------------------------------------------------


class Data:
    """Attribute bag with PyG's ``clone``/``num_nodes``/``num_features``."""

    def __init__(self, **kwargs):
        for k, v in kwargs.items():
            setattr(self, k, v)

    def keys(self):
        return [k for k in self.__dict__ if not k.startswith("_")]

    @property
    def num_nodes(self):
        x = self.__dict__.get("x")
        if x is not None:
            return x.shape[0]
        pos = self.__dict__.get("pos")
        return None if pos is None else pos.shape[0]

    @property
    def num_features(self):
        x = self.__dict__.get("x")
        if x is None:
            return 0
        return 1 if x.dim() == 1 else x.shape[-1]

    num_node_features = num_features

    def clone(self):
        return copy.deepcopy(self)

    def to(self, device, non_blocking=False):
        for k, v in list(self.__dict__.items()):
            if isinstance(v, torch.Tensor):
                setattr(self, k, v.to(device, non_blocking=non_blocking))
        return self


class Batch(Data):
    @property
    def num_graphs(self):
        b = self.__dict__.get("batch")
        return 0 if b is None else int(b.max()) + 1

    @classmethod
    def from_data_list(cls, data_list):
        """PyG ``Collater``: cat along dim 0 (``*index*`` keys along -1 with
        the running node count added), ``batch``/``ptr`` vectors, non-tensor
        attributes gathered into lists."""
        out = cls()
        keys = []
        for d in data_list:
            for k in d.keys():
                if k not in keys:
                    keys.append(k)
        offsets = [0]
        for d in data_list:
            offsets.append(offsets[-1] + d.num_nodes)
        for k in keys:
            vals = [d.__dict__.get(k) for d in data_list]
            if all(isinstance(v, torch.Tensor) for v in vals):
                if "index" in k:
                    vals = [v + offsets[i] for i, v in enumerate(vals)]
                    setattr(out, k, torch.cat(vals, dim=-1))
                else:
                    setattr(out, k, torch.cat([v if v.dim() > 0 else v.view(1) for v in vals], dim=0))
            elif all(v is None for v in vals):
                setattr(out, k, None)
            else:
                setattr(out, k, vals)
        sizes = [d.num_nodes for d in data_list]
        out.batch = torch.repeat_interleave(torch.arange(len(data_list)), torch.tensor(sizes))
        out.ptr = torch.tensor(offsets)
        return out
