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
* Batches holding a non-finite ``x`` or ``edge_attr`` entry (flagged per graph
  when the store is packed) run the reference forward on the layer API with
  the attention computed (``layered.ginet_forward``): the reference's softmax
  turns a non-finite logit into NaN (ginet.py:48-54), and those NaN rows,
  dropped by the depth-0 ``scatter_max`` and propagated by ``max_pool_x``,
  decide which outputs and gradients are NaN.

Differences from the reference, by design: the input batch is not mutated
(the reference overwrites ``data.x`` and offsets ``data.cluster0/1`` in
place); the dropout mask comes from a device counter hash, not the CPU RNG; a
logit that overflows to inf from finite inputs is not detected.  There is no
CPU path: the model must live on the GPU.
"""

from __future__ import annotations

import math

import torch
from torch import nn

from deeprank2_amd import _lib, layered, ops
from deeprank2_amd.fused import BatchHandle, Dropout, FusedFn, FusedSpec, make_pass, resolve_batch, run_pass  # noqa: F401


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
        rowptr, _, col_s = ops.graph_csr(edge_index, n)
        z = ops.spmm_csr(rowptr, col_s, ops.linear_xwT(x, w), n)
        ctx.save_for_backward(x, edge_index, w)
        ctx.dead = (w_ea, w_att)
        return z

    @staticmethod
    def backward(ctx, dz):
        x, edge_index, w = ctx.saved_tensors
        n = x.shape[0]
        trowptr, _, tcol = ops.graph_csr(edge_index, n, transpose=True)
        dy = ops.spmm_csr(trowptr, tcol, dz.contiguous(), n)
        dx = ops.linear_xw(dy, w) if ctx.needs_input_grad[0] else None
        dw = ops.linear_dw(dy, x) if ctx.needs_input_grad[2] else None
        w_ea, w_att = ctx.dead
        return dx, None, dw, torch.zeros_like(w_ea), torch.zeros_like(w_att)


def _attention_conv(layer, x, edge_index, ea):
    """ginet.py:40-60 op for op on the device, attention included: a
    non-finite logit makes ``softmax(dim=1)`` NaN, so its row of ``z`` is NaN
    and the attention weights get NaN (not zero) gradients, as in the
    reference.  Used only when ``x`` or ``edge_attr`` holds a non-finite
    value; for finite inputs the attention is identically 1 and ``_ConvFn``
    runs."""
    row, col = edge_index[0], edge_index[1]
    xcol = nn.functional.linear(x[col], layer.fc.weight)
    xrow = nn.functional.linear(x[row], layer.fc.weight)
    ed = nn.functional.linear(ea, layer.fc_edge_attr.weight)
    logit = nn.functional.leaky_relu(nn.functional.linear(torch.cat([xrow, xcol, ed], dim=1), layer.fc_attention.weight))
    alpha = torch.softmax(logit, dim=1)
    z = torch.zeros(x.shape[0], layer.out_channels, dtype=alpha.dtype, device=alpha.device)
    return z.index_add(0, row, alpha * xcol)


class GINetConvLayer(nn.Module):
    """ginet.py:13-63: ``z_i = sum_{e=(i->j)} softmax_1(att_e) * W x_j``, with
    ``softmax_1 == 1`` for finite logits; ``fc_edge_attr``/``fc_attention``
    exist (and are trained with zero gradients) exactly as in the reference.
    Non-finite inputs take ``_attention_conv`` (NaN rows where the reference
    has them)."""

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
        ops.check_edge_range(edge_index, x.shape[0])
        ea = edge_attr.unsqueeze(-1) if edge_attr.dim() == 1 else edge_attr
        if ea.shape[0] != edge_index.shape[1] or ea.shape[1] != self.fc_edge_attr.in_features:
            msg = f"edge_attr must be [E, {self.fc_edge_attr.in_features}]"
            raise ValueError(msg)
        if not bool(torch.isfinite(x).all()) or not bool(torch.isfinite(ea).all()):
            return _attention_conv(self, x, edge_index, ea)
        return _ConvFn.apply(x, edge_index, self.fc.weight, self.fc_edge_attr.weight, self.fc_attention.weight)

    def __repr__(self):
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels})"


# ---------------------------------------------------------------------------
# Fused per-graph path (dr_ginet_graph_pass + dr_reduce_update)
# ---------------------------------------------------------------------------

PARAM_NAMES = [
    "conv1.fc.weight", "conv1.fc_edge_attr.weight", "conv1.fc_attention.weight",
    "conv2.fc.weight", "conv2.fc_edge_attr.weight", "conv2.fc_attention.weight",
    "conv1_ext.fc.weight", "conv1_ext.fc_edge_attr.weight", "conv1_ext.fc_attention.weight",
    "conv2_ext.fc.weight", "conv2_ext.fc_edge_attr.weight", "conv2_ext.fc_attention.weight",
    "fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias",
]  # fmt: skip


def slab_stride(f):
    """Per-graph conv gradient partials: [W1;W1e] (32 x F), then [W2 | W2e] (1024)."""
    return 32 * f + 1024


def head_stride(out):
    """Per-graph head vectors: g (64), dropped fc1 output (128), its grad (128), dout."""
    return 320 + ((out + 3) & ~3)


def recipe(f, out):
    z = (_lib.DR_GRAD_ZERO, 0, 0, 0)  # attention weights: exact zeros (ginet.py:54)
    slab = _lib.DR_GRAD_SLAB
    return [
        (slab, 0, 0, 0), z, z,
        (slab, 32 * f, 0, 0), z, z,
        (slab, 16 * f, 0, 0), z, z,
        (slab, 32 * f + 512, 0, 0), z, z,
        (_lib.DR_GRAD_OUTER, 192, 0, 64), (_lib.DR_GRAD_HEAD, 192, 0, 0),
        (_lib.DR_GRAD_OUTER, 320, 64, 128), (_lib.DR_GRAD_HEAD, 320, 0, 0),
    ]  # fmt: skip


def weights_c(params):
    w = _lib.GinetWeightsC()
    w.w1, w.w1e = params[0].data_ptr(), params[6].data_ptr()
    w.w2, w.w2e = params[3].data_ptr(), params[9].data_ptr()
    w.fc1w, w.fc1b = params[12].data_ptr(), params[13].data_ptr()
    w.fc2w, w.fc2b = params[14].data_ptr(), params[15].data_ptr()
    return w


def _lds(n, e, k0, p1, k1, f, alias, out):
    return _lib.load().dr_ginet_lds_bytes(n, e, f, k0, p1, k1, alias, out)


def _large(h, w, p):
    """Graphs beyond one workgroup's LDS: tile conv1 kernel + per-graph tail (dr_ginet_large_pass)."""
    plan = h.large_plan(p.out_dim, bf16=p.compute_dtype == _lib.DR_DTYPE_BF16)
    lib = _lib.load()
    rc = lib.dr_ginet_large_pass(h.store.cstruct(), h.descs.data_ptr(), h.B, plan.c, w, p, plan.conv_lds, plan.tail_lds, _lib.stream_ptr(h.store.device))
    _lib.check(rc, "dr_ginet_large_pass")


SPEC = FusedSpec(PARAM_NAMES, recipe, slab_stride, head_stride, "dr_ginet_graph_pass", weights_c, _lds, dropout=0.4, large=_large, bf16=True, layers=layered.ginet_forward, attention=True)


def graph_pass(h: BatchHandle, params, out_dim, flags, **kw):
    """One dr_ginet_graph_pass launch (see fused.make_pass for the keywords)."""
    run_pass(SPEC, h, params, make_pass(out_dim, flags, **kw))


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

    fused_spec = SPEC

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
        if layered.needs_layers(SPEC, h, self.output_shape):  # non-finite x / edge_attr: the attention matters
            return SPEC.layers(self, layered.batch_tensors(h), self.training, mask=dropout_mask)
        dropout = None
        if self.training and self.dropout > 0:
            if dropout_mask is not None:
                dropout = Dropout(self.dropout, mask=dropout_mask.to(device=dev, dtype=torch.uint8).contiguous())
            else:
                dropout = self.next_dropout()
        return FusedFn.apply(SPEC, h, dropout, self.output_shape, *params)
