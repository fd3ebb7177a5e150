"""FoutLayer and FoutNet on MI355X — drop-in for ``deeprank2.neuralnets.gnn.foutnet``.

Same constructor signatures, parameter names/shapes/initialisation order and
``state_dict`` keys as the reference (``deeprank2/neuralnets/gnn/foutnet.py:13-118``).

* ``FoutNet.forward(batch)`` runs one HIP workgroup per graph
  (``dr_fout_graph_pass``): conv1 as one GEMM over ``[x | mean_N(x)]``, depth-0
  community pooling, conv2 on the pooled graph, depth-1 max pooling, per-graph
  mean and fc1/relu/fc2, all in LDS; the backward re-runs the pass in
  backward mode and reduces the per-graph partials (``dr_reduce_update``).
* ``FoutLayer.forward(x, edge_index)`` works on any edge list with the
  generic CSR kernels (the reference's per-node Python loop,
  foutnet.py:56-58, becomes one CSR row-mean).

A node without an out-edge gets ``mean(empty) = NaN`` in its neighbour term
exactly as in the reference; the NaN then flows through relu and the pooling
with the reference's semantics (torch_scatter drops it at depth 0, PyG's
amax propagates it at depth 1).  There is no CPU path.
"""

from __future__ import annotations

import math

import torch
from torch import nn

from deeprank2_amd import _lib, layered, ops
from deeprank2_amd.fused import BatchHandle, FusedFn, FusedSpec, make_pass, resolve_batch, run_pass


def _uniform(size, t):
    """torch_geometric.nn.inits.uniform: U(-1/sqrt(size), 1/sqrt(size))."""
    if t is not None:
        bound = 1.0 / math.sqrt(size)
        t.data.uniform_(-bound, bound)


class _FoutLayerFn(torch.autograd.Function):
    """out = x Wc + rowmean_A(x) Wn + b; the gradient into Wn flows only
    through rows with at least one out-edge (the reference's empty mean has no
    inputs to differentiate)."""

    @staticmethod
    def forward(ctx, x, edge_index, wc, wn, bias):
        n = x.shape[0]
        rowptr, _, col = ops.graph_csr(edge_index, n)
        zm = ops.spmm_csr(rowptr, col, x, n, mean=True)
        out = ops.linear_xwT(x, wc.t().contiguous()) + ops.linear_xwT(zm, wn.t().contiguous())
        if bias is not None:
            out = out + bias
        ctx.save_for_backward(x, edge_index, wc, wn, zm, rowptr)
        ctx.has_bias = bias is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        x, edge_index, wc, wn, zm, rowptr = ctx.saved_tensors
        n = x.shape[0]
        dout = dout.contiguous()
        deg = (rowptr[1:] - rowptr[:-1]).to(torch.float32).unsqueeze(1)
        has = deg > 0
        dwc = ops.linear_dw(dout, x).t().contiguous()
        # rows without out-edges contribute nothing: neither their (NaN) mean nor their dout
        dout_has = torch.where(has, dout, torch.zeros_like(dout))
        dwn = ops.linear_dw(dout_has, torch.where(has, zm, torch.zeros_like(zm))).t().contiguous()
        # d(neighbour term) / x_j = sum_{i: i->j} dout_i / deg_i  (transposed CSR)
        trowptr, _, tcol = ops.graph_csr(edge_index, n, transpose=True)
        dbeta = ops.spmm_csr(trowptr, tcol, torch.where(has, dout / deg.clamp_min(1), torch.zeros_like(dout)), n)
        dx = ops.linear_xwT(dout, wc) + ops.linear_xwT(dbeta, wn)
        db = dout.sum(0) if ctx.has_bias else None
        return dx, None, dwc, dwn, db


class FoutLayer(nn.Module):
    """foutnet.py:13-69 (eq. (1) of Fout et al., NIPS 2018)."""

    def __init__(self, in_channels: int, out_channels: int, bias: bool = True):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.wc = nn.Parameter(torch.Tensor(in_channels, out_channels))
        self.wn = nn.Parameter(torch.Tensor(in_channels, out_channels))
        if bias:
            self.bias = nn.Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        size = self.in_channels
        _uniform(size, self.wc)
        _uniform(size, self.wn)
        _uniform(size, self.bias)

    def forward(self, x, edge_index):
        _lib.require_device(x, edge_index)
        ops.check_edge_range(edge_index, x.shape[0])
        return _FoutLayerFn.apply(x.float(), edge_index, self.wc, self.wn, self.bias)

    def __repr__(self):
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels})"


# ---------------------------------------------------------------------------
# Fused per-graph path (dr_fout_graph_pass + dr_reduce_update)
# ---------------------------------------------------------------------------

PARAM_NAMES = [
    "conv1.wc", "conv1.wn", "conv1.bias", "conv2.wc", "conv2.wn", "conv2.bias",
    "fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias",
]  # fmt: skip


def slab_stride(f):
    """dWc1 | dWn1 (F x 16 each) | db1 (16) | dWc2 | dWn2 (16 x 32 each) | db2 (32)."""
    return 32 * f + 1072


def head_stride(out):
    """g (32) | relu(fc1) (64) | its grad (64) | dout."""
    return 160 + ((out + 3) & ~3)


def recipe(f, out):
    slab = _lib.DR_GRAD_SLAB
    return [
        (slab, 0, 0, 0), (slab, 16 * f, 0, 0), (slab, 32 * f, 0, 0),
        (slab, 32 * f + 16, 0, 0), (slab, 32 * f + 528, 0, 0), (slab, 32 * f + 1040, 0, 0),
        (_lib.DR_GRAD_OUTER, 96, 0, 32), (_lib.DR_GRAD_HEAD, 96, 0, 0),
        (_lib.DR_GRAD_OUTER, 160, 32, 64), (_lib.DR_GRAD_HEAD, 160, 0, 0),
    ]  # fmt: skip


def weights_c(params):
    w = _lib.FoutWeightsC()
    w.wc1, w.wn1, w.b1, w.wc2, w.wn2, w.b2, w.fc1w, w.fc1b, w.fc2w, w.fc2b = (p.data_ptr() for p in params)
    return w


def _lds(n, e, k0, p1, k1, f, alias, out):
    return _lib.load().dr_fout_lds_bytes(n, e, f, k0, p1, k1, alias, out)


def _large(h, w, p):
    """Graphs beyond one workgroup's LDS: tile conv1 kernel + per-graph tail (dr_fout_large_pass)."""
    plan = h.large_plan(p.out_dim, kind="fout")
    rc = _lib.load().dr_fout_large_pass(h.store.cstruct(), h.descs.data_ptr(), h.B, plan.c, w, p, plan.zs, plan.conv_lds, plan.tail_lds, _lib.stream_ptr(h.store.device))
    _lib.check(rc, "dr_fout_large_pass")


SPEC = FusedSpec(PARAM_NAMES, recipe, slab_stride, head_stride, "dr_fout_graph_pass", weights_c, _lds, dropout=0.0, large=_large, layers=layered.foutnet_forward)


def graph_pass(h: BatchHandle, params, out_dim, flags, **kw):
    """One dr_fout_graph_pass launch (see fused.make_pass for the keywords)."""
    run_pass(SPEC, h, params, make_pass(out_dim, flags, **kw))


class FoutNet(nn.Module):
    """foutnet.py:72-118 (``input_shape_edge`` is accepted and ignored)."""

    def __init__(self, input_shape, output_shape=1, input_shape_edge=None):  # noqa: ARG002
        super().__init__()
        self.conv1 = FoutLayer(input_shape, 16)
        self.conv2 = FoutLayer(16, 32)
        self.fc1 = nn.Linear(32, 64)
        self.fc2 = nn.Linear(64, output_shape)
        self.clustering = "mcl"
        self.input_shape = input_shape
        self.output_shape = output_shape

    fused_spec = SPEC
    dropout = 0.0

    def ordered_params(self):
        named = dict(self.named_parameters())
        return [named[n] for n in PARAM_NAMES]

    def forward(self, data):
        params = [p.contiguous() for p in self.ordered_params()]
        dev = params[0].device
        if dev.type != "cuda":
            msg = "deeprank2_amd.FoutNet runs on the MI355X only: move the model to a cuda device (no CPU fallback)"
            raise RuntimeError(msg)
        h = resolve_batch(data, dev)
        if h.store.n_feat != self.input_shape:
            msg = f"batch has {h.store.n_feat} node features, model expects {self.input_shape}"
            raise ValueError(msg)
        if layered.needs_layers(SPEC, h, self.output_shape):  # a graph beyond one workgroup's LDS
            return SPEC.layers(self, layered.batch_tensors(h), self.training)
        return FusedFn.apply(SPEC, h, None, self.output_shape, *params)
