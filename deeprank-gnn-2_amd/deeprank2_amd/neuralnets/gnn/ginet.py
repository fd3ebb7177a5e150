"""GINet and GINetConvLayer on MI355X — drop-in for ``deeprank2.neuralnets.gnn.ginet``.

Same constructor signatures, parameter names/shapes/initialisation and
``state_dict`` keys as the reference (``deeprank2/neuralnets/gnn/ginet.py:13-125``),
so reference checkpoints load unchanged and ``Trainer`` builds it with
``neuralnet(num_node_features, output_shape, num_edge_features)``
(``trainer.py:377``).

* ``GINet.forward(batch)`` runs one HIP workgroup per graph
  (``dr_ginet_graph_pass``): conv1 of both branches as one GEMM, CSR
  aggregation, depth-0 community pooling, conv2, depth-1 max pooling, per-graph
  mean and the fc1/relu/dropout/fc2 head, all in LDS.  Its autograd backward
  re-runs the graph pass in backward mode and reduces the per-graph partials
  into the 16 parameter gradients (``dr_ginet_reduce_update``); the attention
  parameters get exact-zero gradients, as in the reference (their softmax is
  over a size-1 dimension, ginet.py:54).
* ``GINetConvLayer.forward(x, edge_index, edge_attr)`` works on any edge list
  (asymmetric, self loops, duplicates) with the generic CSR kernels.

Differences from the reference, by design: the input batch is not mutated
(the reference overwrites ``data.x`` and offsets ``data.cluster0/1`` in
place); the dropout mask comes from torch's device RNG, not the CPU RNG; with
non-finite node features the set of NaN outputs can differ (the reference's
attention turns a non-finite logit into NaN, ginet.py:54).  There is no CPU
path: the model must live on the GPU.
"""

from __future__ import annotations

import math

import numpy as np
import torch
from torch import nn

from deeprank2_amd import _lib, ops
from deeprank2_amd.store import GraphStore, pack_graphs, records_from_batch


def _uniform(size, t):
    """torch_geometric.nn.inits.uniform: U(-1/sqrt(size), 1/sqrt(size))."""
    if t is not None:
        bound = 1.0 / math.sqrt(size)
        t.data.uniform_(-bound, bound)


# ---------------------------------------------------------------------------
# GINetConvLayer (generic kernels)
# ---------------------------------------------------------------------------


class _ConvFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, edge_index, w, w_ea, w_att):
        n = x.shape[0]
        row, col = edge_index[0], edge_index[1]
        rowptr, _, col_s = ops.csr_from_coo(row, col, n)
        z = ops.spmm_csr(rowptr, col_s, ops.linear_xwT(x, w), n)
        ctx.save_for_backward(x, edge_index, w)
        ctx.dead = (w_ea, w_att)
        return z

    @staticmethod
    def backward(ctx, dz):
        x, edge_index, w = ctx.saved_tensors
        n = x.shape[0]
        trowptr, _, tcol = ops.csr_from_coo(edge_index[1], edge_index[0], n)
        dy = ops.spmm_csr(trowptr, tcol, dz.contiguous(), n)
        dx = ops.linear_xw(dy, w) if ctx.needs_input_grad[0] else None
        dw = ops.linear_dw(dy, x) if ctx.needs_input_grad[2] else None
        w_ea, w_att = ctx.dead
        return dx, None, dw, torch.zeros_like(w_ea), torch.zeros_like(w_att)


class GINetConvLayer(nn.Module):
    """ginet.py:13-63: ``z_i = sum_{e=(i->j)} softmax_1(att_e) * W x_j``, with
    ``softmax_1 == 1``; ``fc_edge_attr``/``fc_attention`` exist (and are
    trained with zero gradients) exactly as in the reference."""

    def __init__(self, in_channels, out_channels, number_edge_features=1, bias=False):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.fc = nn.Linear(self.in_channels, self.out_channels, bias=bias)
        self.fc_edge_attr = nn.Linear(number_edge_features, number_edge_features, bias=bias)
        self.fc_attention = nn.Linear(2 * self.out_channels + number_edge_features, 1, bias=bias)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        for lin in (self.fc, self.fc_attention, self.fc_edge_attr):  # ginet.py:34-38 order
            _uniform(self.in_channels, lin.weight)

    def forward(self, x, edge_index, edge_attr):
        if self.fc.bias is not None:
            msg = "GINetConvLayer(bias=True) is not supported on the MI355X path"
            raise NotImplementedError(msg)
        _lib.require_device(x, edge_index)
        if edge_index.numel():
            lo, hi = int(edge_index.min()), int(edge_index.max())
            if lo < 0 or hi >= x.shape[0]:
                msg = f"edge_index out of range [0, {x.shape[0]})"
                raise IndexError(msg)
        ea = edge_attr.unsqueeze(-1) if edge_attr.dim() == 1 else edge_attr
        if ea.shape[0] != edge_index.shape[1] or ea.shape[1] != self.fc_edge_attr.in_features:
            msg = f"edge_attr must be [E, {self.fc_edge_attr.in_features}]"
            raise ValueError(msg)
        return _ConvFn.apply(x, edge_index, self.fc.weight, self.fc_edge_attr.weight, self.fc_attention.weight)

    def __repr__(self):
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels})"


# ---------------------------------------------------------------------------
# Fused per-graph engine
# ---------------------------------------------------------------------------

PARAM_NAMES = [
    "conv1.fc.weight", "conv1.fc_edge_attr.weight", "conv1.fc_attention.weight",
    "conv2.fc.weight", "conv2.fc_edge_attr.weight", "conv2.fc_attention.weight",
    "conv1_ext.fc.weight", "conv1_ext.fc_edge_attr.weight", "conv1_ext.fc_attention.weight",
    "conv2_ext.fc.weight", "conv2_ext.fc_edge_attr.weight", "conv2_ext.fc_attention.weight",
    "fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias",
]  # fmt: skip


def slab_stride(f):
    return 32 * f + 1024


def head_stride(out):
    return 320 + ((out + 3) & ~3)


class BatchHandle:
    """A mini-batch as the kernels see it: a store + graph ids (host and device)."""

    def __init__(self, store: GraphStore, gids_host: np.ndarray):
        self.store = store
        self.gids_host = np.ascontiguousarray(gids_host, dtype=np.int32)
        self.gids = torch.from_numpy(self.gids_host).to(store.device)
        self.descs = store.descriptors(self.gids_host)
        self.B = int(self.gids_host.size)
        self.max_sizes = store.max_sizes(self.gids_host)
        self._lds = {}

    def lds(self, out_dim):
        v = self._lds.get(out_dim)
        if v is None:
            n, e, k0, p1, k1 = self.max_sizes
            v = int(_lib.load().dr_ginet_lds_bytes(n, e, self.store.n_feat, k0, p1, k1, int(self.store.packed.transpose_aliased), out_dim))
            if v > 160 * 1024:
                msg = f"largest graph of the batch needs {v} B of LDS (> 160 KiB): the streamed large-graph path is not built yet"
                raise RuntimeError(msg)
            self._lds[out_dim] = v
        return v


def resolve_batch(data, device) -> BatchHandle:
    """Our DataLoader attaches a handle; any other PyG-style batch is packed here."""
    h = getattr(data, "_dr_handle", None)
    if h is not None:
        return h
    store = GraphStore(pack_graphs(records_from_batch(data)), device)
    return BatchHandle(store, np.arange(store.n_graphs, dtype=np.int32))


def weights_c(params):
    w = _lib.GinetWeightsC()
    w.w1, w.w1e = params[0].data_ptr(), params[6].data_ptr()
    w.w2, w.w2e = params[3].data_ptr(), params[9].data_ptr()
    w.fc1w, w.fc1b = params[12].data_ptr(), params[13].data_ptr()
    w.fc2w, w.fc2b = params[14].data_ptr(), params[15].data_ptr()
    return w


class Dropout:
    """How fc1's output is dropped: ``mask`` (uint8 [B,128] keep mask) or the
    in-kernel counter hash ``(seed, offset)`` with probability ``p``."""

    def __init__(self, p, mask=None, seed=None, offset=0):
        self.p = float(p)
        self.mask = mask
        self.seed = seed
        self.offset = int(offset)

    @property
    def scale(self):
        return 1.0 / (1.0 - self.p)


def graph_pass(h: BatchHandle, params, out_dim, flags, *, dropout: Dropout | None = None, dout=None, loss_kind=_lib.DR_LOSS_NONE, loss_scale=1.0, class_w=None, out=None, loss_per_graph=None, slab=None, head=None, stamps=None):
    dev = h.store.device
    p = _lib.GinetPassC()
    p.flags = flags
    p.out_dim = out_dim
    p.loss_kind = loss_kind
    mask = None
    if dropout is None:
        p.use_dropout = _lib.DR_DROPOUT_OFF
    elif dropout.mask is not None:
        mask = dropout.mask
        p.use_dropout = _lib.DR_DROPOUT_MASK
        p.drop_scale = dropout.scale
    else:
        p.use_dropout = _lib.DR_DROPOUT_HASH
        p.drop_scale = dropout.scale
        p.drop_p = dropout.p
        p.drop_seed = dropout.seed
        p.drop_offset = dropout.offset
    p.loss_scale = loss_scale
    p.mask = _lib.ptr(mask)
    p.class_w = _lib.ptr(class_w)
    p.out = _lib.ptr(out)
    p.dout = _lib.ptr(dout)
    p.loss_per_graph = _lib.ptr(loss_per_graph)
    p.slab = _lib.ptr(slab)
    p.head = _lib.ptr(head)
    p.stamps = _lib.ptr(stamps)
    w = weights_c(params)
    rc = _lib.load().dr_ginet_graph_pass(h.store.cstruct(), h.descs.data_ptr(), h.B, w, p, h.lds(out_dim), _lib.stream_ptr(dev))
    _lib.check(rc, "dr_ginet_graph_pass")


def reduce_update(h: BatchHandle, params, grads, out_dim, slab, head, adam=None, states=None, loss_per_graph=None, loss_scale=1.0, loss_out=None):
    t = _lib.ParamTableC()
    for i, prm in enumerate(params):
        t.param[i] = prm.data_ptr()
        t.grad[i] = None if grads is None or grads[i] is None else grads[i].data_ptr()
        t.numel[i] = prm.numel()
        if states is not None:
            t.exp_avg[i] = states[i][0].data_ptr()
            t.exp_avg_sq[i] = states[i][1].data_ptr()
    a = adam if adam is not None else _lib.AdamC()
    rc = _lib.load().dr_ginet_reduce_update(t, h.store.n_feat, out_dim, _lib.ptr(slab), _lib.ptr(head), h.B, a, _lib.ptr(loss_per_graph), loss_scale, _lib.ptr(loss_out), _lib.stream_ptr(h.store.device))
    _lib.check(rc, "dr_ginet_reduce_update")


class _GINetFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, h, dropout, out_dim, *params):
        out = torch.empty(h.B, out_dim, dtype=torch.float32, device=h.store.device)
        graph_pass(h, params, out_dim, _lib.DR_PASS_FORWARD, dropout=dropout, out=out)
        ctx.h, ctx.dropout, ctx.out_dim = h, dropout, out_dim
        ctx.save_for_backward(*params)
        return out

    @staticmethod
    def backward(ctx, dout):
        params = ctx.saved_tensors
        h, out_dim = ctx.h, ctx.out_dim
        dev = h.store.device
        slab = torch.empty(h.B * slab_stride(h.store.n_feat), dtype=torch.float32, device=dev)
        head = torch.empty(h.B * head_stride(out_dim), dtype=torch.float32, device=dev)
        graph_pass(h, params, out_dim, _lib.DR_PASS_BACKWARD, dropout=ctx.dropout, dout=dout.contiguous(), slab=slab, head=head)
        grads = [torch.empty_like(p) for p in params]
        reduce_update(h, params, grads, out_dim, slab, head)
        return (None, None, None, *grads)


class GINet(nn.Module):
    """ginet.py:66-125 (two-branch GINetConvLayer net with community pooling)."""

    def __init__(self, input_shape, output_shape=1, input_shape_edge=1):
        super().__init__()
        self.conv1 = GINetConvLayer(input_shape, 16, input_shape_edge)
        self.conv2 = GINetConvLayer(16, 32, input_shape_edge)
        self.conv1_ext = GINetConvLayer(input_shape, 16, input_shape_edge)
        self.conv2_ext = GINetConvLayer(16, 32, input_shape_edge)
        self.fc1 = nn.Linear(2 * 32, 128)
        self.fc2 = nn.Linear(128, output_shape)
        self.clustering = "mcl"
        self.dropout = 0.4
        self.input_shape = input_shape
        self.output_shape = output_shape
        self._drop_seed = None
        self._drop_calls = 0

    def ordered_params(self):
        named = dict(self.named_parameters())
        return [named[n] for n in PARAM_NAMES]

    def next_dropout(self):
        """Training-mode dropout of fc1's output (ginet.py:122) drawn by the
        in-kernel counter hash: a fresh (seed, offset) per forward call."""
        if self._drop_seed is None:
            self._drop_seed = int(torch.randint(0, 2**62, (1,)).item())
        self._drop_calls += 1
        return Dropout(self.dropout, seed=self._drop_seed, offset=self._drop_calls)

    def forward(self, data, dropout_mask=None):
        params = [p.contiguous() for p in self.ordered_params()]
        dev = params[0].device
        if dev.type != "cuda":
            msg = "deeprank2_amd.GINet runs on the MI355X only: move the model to a cuda device (no CPU fallback)"
            raise RuntimeError(msg)
        h = resolve_batch(data, dev)
        if h.store.n_feat != self.input_shape:
            msg = f"batch has {h.store.n_feat} node features, model expects {self.input_shape}"
            raise ValueError(msg)
        dropout = None
        if self.training and self.dropout > 0:
            if dropout_mask is not None:
                dropout = Dropout(self.dropout, mask=dropout_mask.to(device=dev, dtype=torch.uint8).contiguous())
            else:
                dropout = self.next_dropout()
        return _GINetFn.apply(h, dropout, self.output_shape, *params)
