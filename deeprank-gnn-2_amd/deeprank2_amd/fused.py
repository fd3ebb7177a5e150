"""Machinery shared by the per-graph fused models (GINet, FoutNet, ...).

* ``BatchHandle``: a mini-batch as the kernels see it — graph ids into an
  HBM-resident ``GraphStore`` plus their 64-byte ``dr_graph_desc`` records
  (this is the whole "collate" of ``trainer.py:541``).
* ``Dropout``: explicit keep mask, or the in-kernel counter hash.
* ``FusedSpec``: what a model contributes — its C graph-pass entry, weight
  struct, per-graph partial layout and the recipe that turns the partials
  into each parameter's gradient (``dr_reduce_update``).
* ``param_table`` / ``reduce_update``: the shared gradient reduction + Adam.
"""

from __future__ import annotations

from dataclasses import dataclass
from typing import Callable

import numpy as np
import torch

from deeprank2_amd import _lib
from deeprank2_amd.store import GraphStore, pack_graphs, records_from_batch


class BatchHandle:
    """A mini-batch: graph ids into a store, with their device descriptors."""

    def __init__(self, store: GraphStore, gids_host: np.ndarray):
        self.store = store
        self.gids_host = np.ascontiguousarray(gids_host, dtype=np.int32)
        self.gids = torch.from_numpy(self.gids_host).to(store.device)
        self.descs = store.descriptors(self.gids_host)
        self.B = int(self.gids_host.size)
        self.max_sizes = store.max_sizes(self.gids_host)
        self._lds = {}

    def lds(self, key, fn):
        """Dynamic LDS bytes for the largest graph of the batch (cached per model kind)."""
        v = self._lds.get(key)
        if v is None:
            v = int(fn(*self.max_sizes))
            if v > 160 * 1024:
                msg = f"largest graph of the batch needs {v} B of LDS (> 160 KiB): the streamed large-graph path is not built yet"
                raise RuntimeError(msg)
            self._lds[key] = v
        return v


def resolve_batch(data, device) -> BatchHandle:
    """Our DataLoader's batches name their graphs in the dataset's resident
    store; any other PyG-style batch is packed here (one upload per call)."""
    h = getattr(data, "_dr_handle", None)
    if h is not None:
        return h
    fn = getattr(data, "dr_handle", None)
    if callable(fn):
        h = fn(device)
        if h is not None:
            return h
    store = GraphStore(pack_graphs(records_from_batch(data)), device)
    return BatchHandle(store, np.arange(store.n_graphs, dtype=np.int32))


class Dropout:
    """``mask`` (uint8 [B,128] keep mask) or the in-kernel counter hash ``(seed, offset)``."""

    def __init__(self, p, mask=None, seed=None, offset=0):
        self.p = float(p)
        self.mask = mask
        self.seed = seed
        self.offset = int(offset)

    @property
    def scale(self):
        return 1.0 / (1.0 - self.p)


@dataclass
class FusedSpec:
    param_names: list
    recipe: Callable  # (F, out) -> [(kind, off1, off2, cols)] per parameter
    slab_stride: Callable  # F -> floats per graph
    head_stride: Callable  # out -> floats per graph
    entry: str  # C graph-pass entry point
    weights: Callable  # params -> ctypes weights struct
    lds: Callable  # (n, e, k0, p1, k1, F, alias, out) -> bytes
    dropout: float = 0.0


def make_pass(out_dim, flags, *, dropout: Dropout | None = None, dout=None, loss_kind=_lib.DR_LOSS_NONE, loss_scale=1.0, class_w=None, out=None, loss_per_graph=None, slab=None, head=None, stamps=None, step_counter=None):
    p = _lib.PassC()
    p.flags = flags
    p.out_dim = out_dim
    p.loss_kind = loss_kind
    if dropout is None:
        p.use_dropout = _lib.DR_DROPOUT_OFF
    elif dropout.mask is not None:
        p.use_dropout = _lib.DR_DROPOUT_MASK
        p.drop_scale = dropout.scale
        p.mask = dropout.mask.data_ptr()
    else:
        p.use_dropout = _lib.DR_DROPOUT_HASH
        p.drop_scale = dropout.scale
        p.drop_p = dropout.p
        p.drop_seed = dropout.seed
        p.drop_offset = dropout.offset
    p.loss_scale = loss_scale
    p.class_w = _lib.ptr(class_w)
    p.out = _lib.ptr(out)
    p.dout = _lib.ptr(dout)
    p.loss_per_graph = _lib.ptr(loss_per_graph)
    p.slab = _lib.ptr(slab)
    p.head = _lib.ptr(head)
    p.stamps = _lib.ptr(stamps)
    p.step_counter = _lib.ptr(step_counter)
    return p


def lds_for(spec: FusedSpec, h: BatchHandle, out_dim):
    alias = int(h.store.packed.transpose_aliased)
    f = h.store.n_feat
    return h.lds((spec.entry, out_dim), lambda n, e, k0, p1, k1: spec.lds(n, e, k0, p1, k1, f, alias, out_dim))


def run_pass(spec: FusedSpec, h: BatchHandle, params, p, w=None):
    """Launch the model's graph pass on the current stream."""
    if w is None:
        w = spec.weights(params)
    fn = getattr(_lib.load(), spec.entry)
    rc = fn(h.store.cstruct(), h.descs.data_ptr(), h.B, w, p, lds_for(spec, h, p.out_dim), _lib.stream_ptr(h.store.device))
    _lib.check(rc, spec.entry)


def param_table(spec: FusedSpec, params, grads, states, n_feat, out_dim):
    t = _lib.ParamTableC()
    recipe = spec.recipe(n_feat, out_dim)
    if len(params) != len(recipe) or len(params) > _lib.DR_MAX_PARAMS:
        msg = "parameter list and gradient recipe disagree"
        raise ValueError(msg)
    for i, prm in enumerate(params):
        t.param[i] = prm.data_ptr()
        t.grad[i] = None if grads is None or grads[i] is None else grads[i].data_ptr()
        t.numel[i] = prm.numel()
        if states is not None:
            t.exp_avg[i] = states[i][0].data_ptr()
            t.exp_avg_sq[i] = states[i][1].data_ptr()
        kind, off1, off2, cols = recipe[i]
        t.recipe[i].kind, t.recipe[i].off1, t.recipe[i].off2, t.recipe[i].cols = kind, off1, off2, cols
    t.n_params = len(params)
    t.slab_stride = spec.slab_stride(n_feat)
    t.head_stride = spec.head_stride(out_dim)
    return t


def reduce_update(table, B, slab, head, device, adam=None, loss_per_graph=None, loss_scale=1.0, loss_out=None):
    a = adam if adam is not None else _lib.AdamC()
    rc = _lib.load().dr_reduce_update(table, _lib.ptr(slab), _lib.ptr(head), B, a, _lib.ptr(loss_per_graph), loss_scale, _lib.ptr(loss_out), _lib.stream_ptr(device))
    _lib.check(rc, "dr_reduce_update")


class FusedFn(torch.autograd.Function):
    """Autograd bridge: forward = graph pass (FORWARD); backward = graph pass
    (BACKWARD, upstream dout) + gradient reduction into every parameter."""

    @staticmethod
    def forward(ctx, spec, h, dropout, out_dim, *params):
        out = torch.empty(h.B, out_dim, dtype=torch.float32, device=h.store.device)
        run_pass(spec, h, params, make_pass(out_dim, _lib.DR_PASS_FORWARD, dropout=dropout, out=out))
        ctx.spec, ctx.h, ctx.dropout, ctx.out_dim = spec, h, dropout, out_dim
        ctx.save_for_backward(*params)
        return out

    @staticmethod
    def backward(ctx, dout):
        params = ctx.saved_tensors
        spec, h, out_dim = ctx.spec, ctx.h, ctx.out_dim
        dev = h.store.device
        f = h.store.n_feat
        slab = torch.empty(h.B * spec.slab_stride(f), dtype=torch.float32, device=dev)
        head = torch.zeros(h.B * spec.head_stride(out_dim), dtype=torch.float32, device=dev)
        run_pass(spec, h, params, make_pass(out_dim, _lib.DR_PASS_BACKWARD, dropout=ctx.dropout, dout=dout.contiguous(), slab=slab, head=head))
        grads = [torch.empty_like(p) for p in params]
        reduce_update(param_table(spec, params, grads, None, f, out_dim), h.B, slab, head, dev)
        return (None, None, None, None, *grads)
