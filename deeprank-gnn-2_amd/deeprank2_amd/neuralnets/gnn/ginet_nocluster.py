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

import torch
from torch import nn

from deeprank2_amd import _lib, layered
from deeprank2_amd.fused import BatchHandle, Dropout, FusedFn, FusedSpec, make_pass, resolve_batch, run_pass
from deeprank2_amd.neuralnets.gnn import ginet as _ginet
from deeprank2_amd.neuralnets.gnn.ginet import GINetConvLayer

__all__ = ["GINet", "GINetConvLayer"]

PARAM_NAMES = _ginet.PARAM_NAMES


def _lds(n, e, k0, p1, k1, f, alias, out):  # noqa: ARG001
    return _lib.load().dr_ginet_nocluster_lds_bytes(n, e, f, out)


SPEC = FusedSpec(PARAM_NAMES, _ginet.recipe, _ginet.slab_stride, _ginet.head_stride, "dr_ginet_nocluster_graph_pass", _ginet.weights_c, _lds, dropout=0.4, layers=layered.ginet_nocluster_forward, attention=True)


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
