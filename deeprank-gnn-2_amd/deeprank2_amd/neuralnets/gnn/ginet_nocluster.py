"""GINet without clustering on MI355X — drop-in for ``deeprank2.neuralnets.gnn.ginet_nocluster``.

Same constructor signature, parameter names/shapes/initialisation order and
``state_dict`` keys as the reference (``deeprank2/neuralnets/gnn/ginet_nocluster.py:12-111``);
``GINetConvLayer`` is the same layer as in ``ginet.py`` and is shared with
:mod:`deeprank2_amd.neuralnets.gnn.ginet`.

``GINet.forward(batch)`` runs one HIP workgroup per graph
(``dr_ginet_nocluster_graph_pass``): both conv branches on the full graph
(aggregate-then-GEMM on MFMA), per-graph mean, fc1/relu/dropout/fc2; the
backward re-runs the pass and reduces per-graph partials with the pooled
GINet's recipe.  No clusters are needed.  There is no CPU path.
"""

from __future__ import annotations

import numpy as np
import torch
from torch import nn

from deeprank2_amd import _lib, layered
from deeprank2_amd.fused import LDS_MAX, BatchHandle, Dropout, FusedFn, FusedSpec, make_pass, resolve_batch, run_pass, vanilla_tile_plan
from deeprank2_amd.neuralnets.gnn import ginet as _ginet
from deeprank2_amd.neuralnets.gnn.ginet import GINetConvLayer

__all__ = ["GINet", "GINetConvLayer"]

PARAM_NAMES = _ginet.PARAM_NAMES


def _lds(n, e, k0, p1, k1, f, alias, out):  # noqa: ARG001
    return _lib.load().dr_ginet_nocluster_lds_bytes(n, e, f, out)


NC_TILE = 64  # rows per tile of the large-graph pipeline (its kernels hold at most 64)


class _NcPlan:
    """Host side of dr_nc_plan for one batch: node rows, the edge-tile plan
    (halos of out- and in-neighbours, as the Vanilla pipeline's) and the scratch."""

    def __init__(self, h: BatchHandle):
        st = h.store
        idx = h.gids_host.astype(np.int64)
        n = st._sizes[0][idx]  # noqa: SLF001
        row0 = np.concatenate([[0], np.cumsum(n)]).astype(np.int32)
        plan = vanilla_tile_plan(h, n, row0, NC_TILE, st.n_edge_feat, lds_check=False)
        if plan is None:
            msg = "ginet_nocluster large-graph path: no tile plan for this batch (a tile's halo exceeds 65535 nodes)"
            raise RuntimeError(msg)
        tensors, (n_tiles, hmax, emax, tmax) = plan
        lib = _lib.load()
        self.lds = int(lib.dr_nc_large_lds_bytes(st.n_feat, hmax, emax, tmax, 16))
        if self.lds > LDS_MAX:
            msg = f"ginet_nocluster large-graph path needs {self.lds} B of LDS (> 160 KiB)"
            raise RuntimeError(msg)
        dev = st.device
        tiles = (n + NC_TILE - 1) // NC_TILE
        ints = torch.from_numpy(np.concatenate([row0, np.repeat(np.arange(h.B, dtype=np.int32), n), np.concatenate([[0], np.cumsum(tiles)]).astype(np.int32)])).to(dev)
        self.buf = torch.empty(max(1, int(lib.dr_nc_large_scratch_floats(int(row0[-1]), h.B, n_tiles, st.n_feat))), dtype=torch.float32, device=dev)
        self.keep = [ints, *tensors]
        c = _lib.NcPlanC()
        base = ints.data_ptr()
        c.base, c.row0, c.row_slot, c.n_rows = self.buf.data_ptr(), base, base + 4 * (h.B + 1), int(row0[-1])
        c.tile_first = base + 4 * (h.B + 1 + int(row0[-1]))
        (c.tile_row0, c.halo_off, c.halo_ids, c.lcol_off, c.lcol, c.ltcol_off, c.ltcol) = (t.data_ptr() for t in tensors)
        c.n_tiles, c.halo_max, c.tile_edges_max, c.tile_tedges_max = n_tiles, hmax, emax, tmax
        self.c = c


def _large(h, w, p):
    """Graphs beyond one workgroup's LDS: the tile-kernel pipeline (dr_ginet_nocluster_large_pass)."""
    plan = h._lds.get("nc_plan")  # noqa: SLF001
    if plan is None:
        plan = h._lds["nc_plan"] = _NcPlan(h)  # noqa: SLF001
    rc = _lib.load().dr_ginet_nocluster_large_pass(h.store.cstruct(), h.descs.data_ptr(), h.B, plan.c, w, p, _lib.stream_ptr(h.store.device))
    _lib.check(rc, "dr_ginet_nocluster_large_pass")


SPEC = FusedSpec(PARAM_NAMES, _ginet.recipe, _ginet.slab_stride, _ginet.head_stride, "dr_ginet_nocluster_graph_pass", _ginet.weights_c, _lds, dropout=0.4, large=_large, layers=layered.ginet_nocluster_forward, attention=True)


def graph_pass(h: BatchHandle, params, out_dim, flags, **kw):
    """One dr_ginet_nocluster_graph_pass launch (see fused.make_pass for the keywords)."""
    run_pass(SPEC, h, params, make_pass(out_dim, flags, **kw))


class GINet(nn.Module):
    """ginet_nocluster.py:66-111."""

    def __init__(self, input_shape, output_shape=1, input_shape_edge=1):
        super().__init__()
        self.conv1 = GINetConvLayer(input_shape, 16, input_shape_edge)
        self.conv2 = GINetConvLayer(16, 32, input_shape_edge)
        self.conv1_ext = GINetConvLayer(input_shape, 16, input_shape_edge)
        self.conv2_ext = GINetConvLayer(16, 32, input_shape_edge)
        self.fc1 = nn.Linear(2 * 32, 128)
        self.fc2 = nn.Linear(128, output_shape)
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
        """Training-mode dropout of fc1's output (ginet_nocluster.py:108), in-kernel counter hash."""
        if self._drop_seed is None:
            self._drop_seed = int(torch.randint(0, 2**62, (1,)).item())
        self._drop_calls += 1
        return Dropout(self.dropout, seed=self._drop_seed, offset=self._drop_calls)

    def forward(self, data, dropout_mask=None):
        params = [p.contiguous() for p in self.ordered_params()]
        dev = params[0].device
        if dev.type != "cuda":
            msg = "deeprank2_amd GINet (no clustering) runs on the MI355X only: move the model to a cuda device (no CPU fallback)"
            raise RuntimeError(msg)
        h = resolve_batch(data, dev, require_clusters=False)
        if h.store.n_feat != self.input_shape:
            msg = f"batch has {h.store.n_feat} node features, model expects {self.input_shape}"
            raise ValueError(msg)
        if layered.needs_layers(SPEC, h, self.output_shape):  # a graph beyond LDS, or non-finite inputs
            return SPEC.layers(self, layered.batch_tensors(h), self.training, mask=dropout_mask)
        dropout = None
        if self.training and self.dropout > 0:
            if dropout_mask is not None:
                dropout = Dropout(self.dropout, mask=dropout_mask.to(device=dev, dtype=torch.uint8).contiguous())
            else:
                dropout = self.next_dropout()
        return FusedFn.apply(SPEC, h, dropout, self.output_shape, *params)
