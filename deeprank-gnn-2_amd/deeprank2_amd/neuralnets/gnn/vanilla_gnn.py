"""VanillaConvolutionalLayer and VanillaNetwork on MI355X — drop-in for
``deeprank2.neuralnets.gnn.vanilla_gnn``.

Same constructor signatures, parameter names/shapes/initialisation order and
``state_dict`` keys as the reference (``deeprank2/neuralnets/gnn/vanilla_gnn.py:10-65``).

``VanillaNetwork.forward(batch)`` runs ``dr_vanilla_graph_pass``: a pipeline
of batch-wide row-parallel HIP kernels runs both layers with the edge MLP
fused into the CSR gather (the E x 32 messages are never materialised),
``scatter_mean``, the graph MLP, the loss and the backward; node-level
intermediates sit in a per-batch HBM scratch.  ``VanillaConvolutionalLayer.forward`` on an arbitrary
edge list runs the same arithmetic through the layer-level C entries
(``dr_edge_mlp_scatter`` / ``_bwd``).  There is no CPU path.
"""

from __future__ import annotations

import numpy as np
import torch
from torch import nn

from deeprank2_amd import _lib, ops
from deeprank2_amd.fused import LDS_MAX, BatchHandle, FusedFn, FusedSpec, make_pass, resolve_batch, run_pass

MESSAGE = 32


def _r4(v):
    return (v + 3) & ~3


class _VanillaLayerFn(torch.autograd.Function):
    """x' = relu(Wn [x | s] + bn),  s_i = sum_{e: src i} relu(We [x_i | x_j | ea_e] + be)."""

    @staticmethod
    def forward(ctx, x, edge_index, ea, we, be, wn, bn):
        n, f = x.shape
        fe = ea.shape[1]
        g = ops.edge_graph(edge_index, n, ea)
        wa, wb = we[:, :f].contiguous(), we[:, f:2 * f].contiguous()
        a = ops.linear_xwT(x, wa)
        b = ops.linear_xwT(x, wb)
        s = ops.edge_mlp_scatter(g, a, b, we, be, f, fe)
        u = ops.linear_xwT(torch.cat([x, s], 1), wn) + bn
        out = torch.relu(u)
        ctx.save_for_backward(x, we, be, wn, a, b, s, out)
        ctx.g, ctx.f, ctx.fe = g, f, fe
        return out

    @staticmethod
    def backward(ctx, dout):
        x, we, be, wn, a, b, s, out = ctx.saved_tensors
        g, f, fe = ctx.g, ctx.f, ctx.fe
        du = torch.where(out <= 0, torch.zeros_like(dout), dout).contiguous()
        dxs = ops.linear_xw(du, wn)  # [dx_direct | ds]
        ds = dxs[:, f:].contiguous()
        d, dp, eap = ops.edge_mlp_scatter_bwd(g, a, b, we, be, f, fe, ds)
        dwa = ops.linear_dw(d, x)
        dwb = ops.linear_dw(dp, x)
        dwc = eap.reshape(-1, MESSAGE, max(fe, 1)).sum(0)[:, :fe]
        dwe = torch.cat([dwa, dwb, dwc], 1)
        dbe = d.sum(0)
        dwn = ops.linear_dw(du, torch.cat([x, s], 1))
        dbn = du.sum(0)
        dx = dxs[:, :f] + ops.linear_xw(d, we[:, :f].contiguous()) + ops.linear_xw(dp, we[:, f:2 * f].contiguous())
        return dx, None, None, dwe, dbe, dwn, dbn


class VanillaConvolutionalLayer(nn.Module):
    """vanilla_gnn.py:10-38."""

    def __init__(self, count_node_features, count_edge_features):
        super().__init__()
        edge_input_size = 2 * count_node_features + count_edge_features
        self._edge_mlp = nn.Sequential(nn.Linear(edge_input_size, MESSAGE), nn.ReLU())
        self._node_mlp = nn.Sequential(nn.Linear(count_node_features + MESSAGE, count_node_features), nn.ReLU())

    def forward(self, node_features, edge_node_indices, edge_features):
        _lib.require_device(node_features, edge_node_indices, edge_features)
        ea = edge_features.float().reshape(edge_node_indices.shape[1], -1).contiguous()
        e, n = self._edge_mlp[0], self._node_mlp[0]
        return _VanillaLayerFn.apply(node_features.float().contiguous(), edge_node_indices, ea, e.weight, e.bias, n.weight, n.bias)


# ---------------------------------------------------------------------------
# Fused path (dr_vanilla_graph_pass + dr_reduce_update)
# ---------------------------------------------------------------------------

PARAM_NAMES = [
    "_external1._edge_mlp.0.weight", "_external1._edge_mlp.0.bias", "_external1._node_mlp.0.weight", "_external1._node_mlp.0.bias",
    "_external2._edge_mlp.0.weight", "_external2._edge_mlp.0.bias", "_external2._node_mlp.0.weight", "_external2._node_mlp.0.bias",
    "_graph_mlp.0.weight", "_graph_mlp.0.bias", "_graph_mlp.2.weight", "_graph_mlp.2.bias",
]  # fmt: skip


def make_spec(f, fe):
    """The fused spec of a VanillaNetwork(f, out, fe) (partial layouts depend on F and Fe)."""
    ke, kn = 2 * f + fe, f + MESSAGE
    layer = 32 * ke + 32 + f * kn + f
    xs = _r4(f)

    def slab_stride(_f):
        return MAX_SPLIT * 2 * layer  # room for one partial row per workgroup of a split graph

    def head_stride(out):
        return 2 * xs + 256 + _r4(out)  # g | h | dh | dout | d mean

    def recipe(_f, _out):
        sl = _lib.DR_GRAD_SLAB
        rec = []
        for base in (0, layer):
            rec += [(sl, base, 0, 0), (sl, base + 32 * ke, 0, 0), (sl, base + 32 * ke + 32, 0, 0), (sl, base + 32 * ke + 32 + f * kn, 0, 0)]
        rec += [(_lib.DR_GRAD_OUTER, xs + 128, 0, f), (_lib.DR_GRAD_HEAD, xs + 128, 0, 0), (_lib.DR_GRAD_OUTER, xs + 256, xs, 128), (_lib.DR_GRAD_HEAD, xs + 256, 0, 0)]
        return rec

    def weights(params):
        w = _lib.VanillaWeightsC()
        (w.we1, w.be1, w.wn1, w.bn1, w.we2, w.be2, w.wn2, w.bn2, w.g1w, w.g1b, w.g2w, w.g2b) = (p.data_ptr() for p in params)
        return w

    def run(h, w, p, wpack=None):
        st = h.store
        if st.n_edge_feat != fe or st.n_feat != f:
            msg = f"batch has F={st.n_feat}, Fe={st.n_edge_feat}; the model expects F={f}, Fe={fe}"
            raise ValueError(msg)
        lib = _lib.load()
        if fused_fits(h, f, fe):  # split_k(h) workgroups per graph, graph in LDS
            buf, offs, sync, own = h.vanilla_fused_scratch()
            if wpack is None:  # the pass packs the weights into the batch's own copy first
                wpack = own
            else:  # the caller's copy is current (FusedTrainStep: Adam keeps it so, and clears the fault flag)
                p = _lib.PassC.from_buffer_copy(p)
                p.flags |= _lib.DR_PASS_WPACK_CURRENT
            lds = h.lds(("vanilla_fused", fe), lambda n, e, *_: lib.dr_vanilla_fused_lds_bytes(n, e, fe))
            _lib.check(lib.dr_vanilla_fused_pass(st.cstruct(), h.descs.data_ptr(), h.B, w, p, buf.data_ptr(), offs.data_ptr(), split_k(h, f, fe), sync.data_ptr(), wpack.data_ptr(), lds, _lib.stream_ptr(st.device)), "dr_vanilla_fused_pass")
            return
        _pipeline(h, w, p)

    def packed(params):
        """FusedTrainStep's packed weight copy (dr_vanilla_wpack) and its Adam
        mirror map: packing weights that hold 1 + their flat index yields each
        slot's source element; element i's (at most 4) slots go to
        mirror_idx[4i .. 4i+3], -1 padded."""
        lib = _lib.load()
        dev = params[0].device
        stream = _lib.stream_ptr(dev)
        numel = [q.numel() for q in params]
        n = int(lib.dr_vanilla_wpack_floats())
        probe = torch.arange(1, sum(numel) + 1, dtype=torch.float32, device=dev)
        views = [v.view_as(q) for v, q in zip(torch.split(probe, numel), params)]
        tmp = torch.empty(n, dtype=torch.float32, device=dev)
        _lib.check(lib.dr_vanilla_wpack(weights(views), f, fe, tmp.data_ptr(), stream), "dr_vanilla_wpack")
        src = tmp.round().to(torch.int64) - 1
        slot = torch.nonzero(src >= 0).flatten()
        el = src[slot]
        order = torch.argsort(el, stable=True)
        el, slot = el[order], slot[order]
        j = torch.arange(el.numel(), device=dev) - torch.searchsorted(el, el)  # rank among the element's slots
        if el.numel() and int(j.max()) > 3:
            msg = "a weight element appears in more than 4 packed slots"
            raise RuntimeError(msg)
        idx = torch.full((sum(numel), 4), -1, dtype=torch.int32, device=dev)
        idx[el, j] = slot.to(torch.int32)
        buf = torch.empty(n, dtype=torch.float32, device=dev)

        def refresh():
            _lib.check(lib.dr_vanilla_wpack(weights(params), f, fe, buf.data_ptr(), _lib.stream_ptr(dev)), "dr_vanilla_wpack")

        refresh()
        return buf, idx.reshape(-1), refresh

    def _pipeline(h, w, p):
        st = h.store
        lib = _lib.load()
        sc, _keep = h.vanilla_scratch(f, fe)
        lds = int(lib.dr_vanilla_lds_bytes(f, fe, p.out_dim))
        _lib.check(lib.dr_vanilla_graph_pass(st.cstruct(), h.descs.data_ptr(), h.B, w, p, sc, lds, _lib.stream_ptr(st.device)), "dr_vanilla_graph_pass")

    return FusedSpec(PARAM_NAMES, recipe, slab_stride, head_stride, "dr_vanilla_graph_pass", weights, lambda *_: 0, dropout=0.0, run=run, slab_rows=MAX_SPLIT, slab_k=lambda h: split_k(h, f, fe), handoffs=True, wpack=packed)


FUSED_MAX_FE = 4  # vanilla_graph.hip MAXFE
MAX_SPLIT = 4  # DR_VANILLA_MAX_SPLIT
_CUS = {}


def _cus(device):
    """Compute units of the device (256 on a whole MI355X; fewer in a partition
    mode): the per-graph kernel holds one 1024-thread workgroup per CU."""
    key = str(device)
    if key not in _CUS:
        try:
            _CUS[key] = int(torch.cuda.get_device_properties(torch.device(device)).multi_processor_count)
        except (RuntimeError, AssertionError, ValueError):
            _CUS[key] = 256
    return _CUS[key]


def split_k(h: BatchHandle, f, fe):
    """Workgroups per graph of the per-graph kernel for this batch (1 on the
    pipeline): as many as keep the grid within one workgroup per CU (a batch of
    64 graphs on 256 CUs: 4), ``h.vanilla_split`` if set."""
    if not fused_fits(h, f, fe):
        return 1
    if h.vanilla_split is not None:
        k = int(h.vanilla_split)
        if not 1 <= k <= MAX_SPLIT:
            msg = f"vanilla_split must be in 1..{MAX_SPLIT} (got {k})"
            raise ValueError(msg)
        return k
    return max(1, min(MAX_SPLIT, _cus(h.store.device) // max(1, ((h.B + 7) // 8) * 8)))


def fused_fits(h: BatchHandle, f, fe):
    """True when the batch runs on the per-graph fused kernel (dr_vanilla_fused_pass):
    F <= 32, Fe <= 4 and the largest graph's CSR, transpose and node arrays fit
    160 KiB of LDS; otherwise the batch-wide pipeline (dr_vanilla_graph_pass).
    ``h.vanilla_pipeline = True`` forces the pipeline."""
    if getattr(h, "vanilla_pipeline", False) or f > 32 or fe > FUSED_MAX_FE:  # noqa: PLR2004
        return False
    lib = _lib.load()
    return h.lds(("vanilla_fused", fe), lambda n, e, *_: lib.dr_vanilla_fused_lds_bytes(n, e, fe)) <= LDS_MAX


def graph_pass(model, h: BatchHandle, params, out_dim, flags, **kw):
    run_pass(model.fused_spec, h, params, make_pass(out_dim, flags, **kw))


class VanillaNetwork(nn.Module):
    """vanilla_gnn.py:41-65 (no clusters needed)."""

    def __init__(self, input_shape: int, output_shape: int, input_shape_edge: int):
        super().__init__()
        self._external1 = VanillaConvolutionalLayer(input_shape, input_shape_edge)
        self._external2 = VanillaConvolutionalLayer(input_shape, input_shape_edge)
        hidden_size = 128
        self._graph_mlp = nn.Sequential(nn.Linear(input_shape, hidden_size), nn.ReLU(), nn.Linear(hidden_size, output_shape))
        self.input_shape = input_shape
        self.output_shape = output_shape
        self.input_shape_edge = input_shape_edge
        self.fused_spec = make_spec(input_shape, input_shape_edge)

    dropout = 0.0

    def ordered_params(self):
        named = dict(self.named_parameters())
        return [named[n] for n in PARAM_NAMES]

    def forward(self, data):
        params = [p.contiguous() for p in self.ordered_params()]
        dev = params[0].device
        if dev.type != "cuda":
            msg = "deeprank2_amd.VanillaNetwork runs on the MI355X only: move the model to a cuda device (no CPU fallback)"
            raise RuntimeError(msg)
        h = resolve_batch(data, dev, require_clusters=False)
        return FusedFn.apply(self.fused_spec, h, None, self.output_shape, *params)
