"""SGraphAttentionLayer and SGAT on MI355X — drop-in for ``deeprank2.neuralnets.gnn.sgat``.

Same constructor signatures, parameter names/shapes/initialisation order and
``state_dict`` keys as the reference (``deeprank2/neuralnets/gnn/sgat.py:13-133``).

* ``SGAT.forward(batch)`` runs one HIP workgroup per graph
  (``dr_sgat_graph_pass``, the FoutNet kernel family): conv1 as one MFMA GEMM
  over ``[c_i x_i | sum_e a_e x_j / deg_i]`` with ``c_i = sum_e a_e / deg_i``
  (``deg`` clamped to 1, torch_scatter's ``scatter_mean``), depth-0 community
  pooling, conv2 on the pooled graph with the pooled edge_attr (``pool_edge``
  sums, precomputed in the store), depth-1 max pooling, per-graph mean and
  fc1/relu/fc2; backward re-runs the pass and reduces per-graph partials.
* ``SGraphAttentionLayer.forward(x, edge_index, edge_attr)`` works on any
  edge list with the generic kernels (``dr_spmm_csr_w``, ``dr_linear_*``),
  ``undirected=False`` included.

Both need one edge feature (``edge_attr`` [E] or [E, 1]): the reference
multiplies ``edge_attr [E, Fe]`` into ``[E, out]`` (sgat.py:71), which only
broadcasts for Fe = 1 across both layers.  There is no CPU path.
"""

from __future__ import annotations

import math

import torch
from torch import nn

from deeprank2_amd import _lib, layered, ops
from deeprank2_amd.fused import BatchHandle, FusedFn, FusedSpec, make_pass, resolve_batch, run_pass
from deeprank2_amd.neuralnets.gnn import foutnet


def _uniform(size, t):
    if t is not None:
        bound = 1.0 / math.sqrt(size)
        t.data.uniform_(-bound, bound)


class _WSpmm(torch.autograd.Function):
    """out[i] = sum_{e in row i} w_e y[col_e]; dy via the transposed CSR."""

    @staticmethod
    def forward(ctx, y, g, w, tw):
        y = y.contiguous()
        out = torch.empty(g.n, y.shape[1], dtype=torch.float32, device=y.device)
        _lib.check(_lib.load().dr_spmm_csr_w(g.rowptr.data_ptr(), g.col.data_ptr(), w.data_ptr(), y.data_ptr(), g.n, y.shape[1], 0, out.data_ptr(), _lib.stream_ptr(y.device)), "dr_spmm_csr_w")
        ctx.g, ctx.tw = g, tw
        return out

    @staticmethod
    def backward(ctx, dout):
        g, tw = ctx.g, ctx.tw
        dout = dout.contiguous()
        dy = torch.empty(g.n, dout.shape[1], dtype=torch.float32, device=dout.device)
        _lib.check(_lib.load().dr_spmm_csr_w(g.trowptr.data_ptr(), g.tcol.data_ptr(), tw.data_ptr(), dout.data_ptr(), g.n, dout.shape[1], 0, dy.data_ptr(), _lib.stream_ptr(dout.device)), "dr_spmm_csr_w")
        return dy, None, None, None


class _MatMul(torch.autograd.Function):
    """x [M,K] @ W [K,N] on the linear kernels."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return ops.linear_xwT(x.contiguous(), w.t().contiguous())

    @staticmethod
    def backward(ctx, dout):
        x, w = ctx.saved_tensors
        dout = dout.contiguous()
        return ops.linear_xwT(dout, w.contiguous()), ops.linear_dw(dout, x.contiguous()).t()


class SGraphAttentionLayer(nn.Module):
    """sgat.py:13-84: ``z_i = 1/N_i sum_j a_ij [x_i | x_j] W + b``."""

    def __init__(self, in_channels: int, out_channels: int, bias: bool = True, undirected: bool = True):
        super().__init__()
        self.in_channels = in_channels
        self.out_channels = out_channels
        self.undirected = undirected
        self.weight = nn.Parameter(torch.Tensor(2 * in_channels, out_channels))
        if bias:
            self.bias = nn.Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        size = 2 * self.in_channels
        _uniform(size, self.weight)
        _uniform(size, self.bias)

    def forward(self, x, edge_index, edge_attr):
        _lib.require_device(x, edge_index, edge_attr)
        n = x.shape[0]
        ops.check_edge_range(edge_index, n)
        ea = edge_attr.unsqueeze(-1) if edge_attr.dim() == 1 else edge_attr
        if ea.shape[1] != 1:
            msg = f"SGraphAttentionLayer needs one edge feature (edge_attr [E] or [E, 1], got {tuple(edge_attr.shape)}): sgat.py:71 multiplies it into every output channel"
            raise ValueError(msg)
        x = x.float()
        a = ea[:, 0].float().detach()
        fin = self.in_channels
        wt, wb = self.weight[:fin], self.weight[fin:]
        ones = torch.ones(n, 1, dtype=torch.float32, device=x.device)
        # scatter_mean over edge_index[0] into zeros (sgat.py:74-75)
        g = ops.edge_graph(edge_index, n, a.unsqueeze(1))
        w, tw = g.ea[:, 0].contiguous(), g.ea[:, 0][g.teid.long()].contiguous()
        deg = (g.rowptr[1:] - g.rowptr[:-1]).clamp_min(1).to(torch.float32).unsqueeze(1)
        c = _WSpmm.apply(ones, g, w, tw) / deg
        zw = _WSpmm.apply(x, g, w, tw) / deg
        out = _MatMul.apply(c * x, wt) + _MatMul.apply(zw, wb)
        if not self.undirected:
            # second scatter_mean over edge_index[1] into the same out (sgat.py:80-81):
            # out <- (out + sum_{e: col=i} a_e [x_row | x_i] W) / max(cnt_col_i, 1)
            gt = ops.edge_graph(torch.stack([edge_index[1], edge_index[0]]), n, a.unsqueeze(1))
            wt_, twt = gt.ea[:, 0].contiguous(), gt.ea[:, 0][gt.teid.long()].contiguous()
            cnt = (gt.rowptr[1:] - gt.rowptr[:-1]).clamp_min(1).to(torch.float32).unsqueeze(1)
            s_in = _WSpmm.apply(ones, gt, wt_, twt)
            t_in = _WSpmm.apply(x, gt, wt_, twt)
            out = (out + _MatMul.apply(t_in, wt) + _MatMul.apply(s_in * x, wb)) / cnt
        if self.bias is not None:
            out = out + self.bias
        return out

    def __repr__(self):
        return f"{self.__class__.__name__}({self.in_channels}, {self.out_channels})"


# ---------------------------------------------------------------------------
# Fused per-graph path (dr_sgat_graph_pass + dr_reduce_update)
# ---------------------------------------------------------------------------

PARAM_NAMES = ["conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias", "fc1.weight", "fc1.bias", "fc2.weight", "fc2.bias"]


def recipe(f, out):
    """FoutNet's partial layout: d conv*.weight = the dWc|dWn block pair."""
    r = foutnet.recipe(f, out)
    return [r[0], r[2], r[3], r[5], r[6], r[7], r[8], r[9]]


def weights_c(params):
    w1, b1, w2, b2, f1w, f1b, f2w, f2b = params
    fin = w1.shape[0] // 2
    w = _lib.FoutWeightsC()
    w.wc1, w.wn1, w.b1 = w1.data_ptr(), w1.data_ptr() + 4 * fin * 16, b1.data_ptr()
    w.wc2, w.wn2, w.b2 = w2.data_ptr(), w2.data_ptr() + 4 * 16 * 32, b2.data_ptr()
    w.fc1w, w.fc1b, w.fc2w, w.fc2b = f1w.data_ptr(), f1b.data_ptr(), f2w.data_ptr(), f2b.data_ptr()
    return w


def _lds(n, e, k0, p1, k1, f, alias, out):
    return _lib.load().dr_sgat_lds_bytes(n, e, f, k0, p1, k1, alias, out)


def _large(h, w, p):
    """Graphs beyond one workgroup's LDS: tile conv1 kernel + per-graph tail (dr_sgat_large_pass)."""
    plan = h.large_plan(p.out_dim, kind="sgat")
    rc = _lib.load().dr_sgat_large_pass(h.store.cstruct(), h.descs.data_ptr(), h.B, plan.c, w, p, plan.zs, plan.conv_lds, plan.tail_lds, _lib.stream_ptr(h.store.device))
    _lib.check(rc, "dr_sgat_large_pass")


SPEC = FusedSpec(PARAM_NAMES, recipe, foutnet.slab_stride, foutnet.head_stride, "dr_sgat_graph_pass", weights_c, _lds, dropout=0.0, large=_large, layers=layered.sgat_forward)


def graph_pass(h: BatchHandle, params, out_dim, flags, **kw):
    """One dr_sgat_graph_pass launch (see fused.make_pass for the keywords)."""
    run_pass(SPEC, h, params, make_pass(out_dim, flags, **kw))


class SGAT(nn.Module):
    """sgat.py:87-133 (``input_shape_edge`` is accepted and ignored, as in the reference)."""

    def __init__(self, input_shape, output_shape=1, input_shape_edge=None):  # noqa: ARG002
        super().__init__()
        self.conv1 = SGraphAttentionLayer(input_shape, 16)
        self.conv2 = SGraphAttentionLayer(16, 32)
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
            msg = "deeprank2_amd.SGAT runs on the MI355X only: move the model to a cuda device (no CPU fallback)"
            raise RuntimeError(msg)
        h = resolve_batch(data, dev)
        if h.store.n_feat != self.input_shape:
            msg = f"batch has {h.store.n_feat} node features, model expects {self.input_shape}"
            raise ValueError(msg)
        if h.store.n_edge_feat != 1:
            msg = f"SGAT needs exactly one edge feature (got {h.store.n_edge_feat}): sgat.py:71 multiplies edge_attr into every channel"
            raise ValueError(msg)
        if layered.needs_layers(SPEC, h, self.output_shape):  # a graph beyond one workgroup's LDS
            return SPEC.layers(self, layered.batch_tensors(h), self.training)
        return FusedFn.apply(SPEC, h, None, self.output_shape, *params)
