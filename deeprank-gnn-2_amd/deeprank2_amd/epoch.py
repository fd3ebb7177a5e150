"""A whole training epoch of fused steps as ONE captured HIP graph.

``Trainer._epoch`` (reference ``deeprank2/trainer.py:666-724``) walks the
loader's mini-batches and, per batch, builds its descriptors on the host,
copies them to the device, launches the graph pass and the reduce/Adam
kernel, and clones the outputs: tens of microseconds of host work and
launches around a ~20 us step.  ``EpochRunner`` removes all of it from the
epoch loop:

* every graph's 64-byte descriptor sits in a device table built once per
  store; an epoch's batches are one pinned host->device copy of the epoch's
  graph order and one gather (``index_select``) into a fixed descriptor
  buffer that the handles of the epoch's batches view;
* the steps of one epoch (graph pass + reduce/Adam per batch, each writing its
  predictions and loss straight into epoch buffers) are captured once into a
  HIP graph and replayed every epoch: one graph launch per epoch;
* the dropout offset and Adam's step live in FusedTrainStep's device counter,
  so replays advance them exactly as eager steps do.

The launches are the eager steps' launches with the same arguments, except the
dynamic LDS each reserves (sized for the dataset's largest graph rather than
the batch's), so losses, outputs and parameters are bit-identical to eager
steps (``tests/test_gpu_trainer.py``).  Eligible: one process (no process
group), fp32, the model's per-graph kernel holding every graph of the dataset,
no non-finite inputs, MSE or unweighted cross-entropy (the loss scale then
depends only on the batch size).
"""

from __future__ import annotations

import numpy as np
import torch

from deeprank2_amd import _lib
from deeprank2_amd.fused import LDS_MAX, BatchHandle, lds_for, sibling_k


def _static_handle(store, descs, b, max_sizes):
    """A BatchHandle over a fixed descriptor buffer (its graphs change between
    replays; everything sized from it is sized for the dataset's largest graph)."""
    h = BatchHandle.__new__(BatchHandle)
    h.store = store
    h.gids_host = np.zeros(b, dtype=np.int32)  # placeholder: no eligible path reads the ids on the host
    h.gids = None
    h.descs = descs
    h.B = int(b)
    h.max_sizes = max_sizes
    h.nonfinite = False
    h._lds = {}  # noqa: SLF001
    h.force_large = h.force_layers = h.large_onepass = h.mixed_dispatch = False
    h.large_tile = h.vanilla_split = h.fault = None
    h.large_halos = h.large_atomic_max = h.vanilla_words = True
    h.vanilla_tile_rows = 0
    h.sibling_split = 0
    return h


def descriptor_table(store):
    """Every graph's dr_graph_desc on the device, [G, 64] uint8 (built once per store)."""
    t = getattr(store, "_dr_desc_table", None)
    if t is None:
        t = store.descriptors(np.arange(store.packed.n_graphs, dtype=np.int32)).view(-1, 64)
        store._dr_desc_table = t  # noqa: SLF001
    return t


def eligible(step, store) -> bool:
    spec = step.spec
    if step.pg is not None or step.compute_dtype != "f32" or spec.run is not None or step.fuse_update:
        return False
    if step.loss == "ce" and step.class_weights is not None:
        return False
    nf = store.packed.nonfinite
    if nf is not None and bool(np.asarray(nf).any()):
        return False
    probe = _static_handle(store, None, 1, store.max_sizes(np.arange(store.packed.n_graphs)))
    return lds_for(spec, probe, step.out_dim) <= LDS_MAX and sibling_k(spec, probe) == 1


class EpochRunner:
    """The fused steps of one epoch's batches (sizes ``sizes``, in order) as one HIP graph."""

    def __init__(self, step, store, sizes):
        self.step, self.store = step, store
        self.sizes = [int(s) for s in sizes]
        self.offs = np.concatenate([[0], np.cumsum(self.sizes)]).astype(np.int64)
        n, dev = int(self.offs[-1]), step.device
        self.table = descriptor_table(store)
        self.pin = torch.empty(n, dtype=torch.int64, pin_memory=True)
        self.gids = torch.empty(n, dtype=torch.int64, device=dev)
        self.descs = torch.empty(n, 64, dtype=torch.uint8, device=dev)
        ms = store.max_sizes(np.arange(store.packed.n_graphs))
        self.handles = [_static_handle(store, self.descs[o : o + b].view(-1), b, ms) for o, b in zip(self.offs[:-1], self.sizes)]
        self.out = torch.empty(n, step.out_dim, dtype=torch.float32, device=dev)
        self.loss = torch.empty(len(self.sizes), dtype=torch.float32, device=dev)
        self.graph = None
        step._ensure(max(self.sizes))  # noqa: SLF001  (buffers sized before the capture)

    def _steps(self):
        """The epoch's steps, each writing its predictions and loss straight
        into the epoch buffers (the graph pass's ``dr_pass.out`` and the
        reduce's loss pointer redirected per step: no copy launches)."""
        s = self.step
        passes = (s._pass, s._pass_nodrop)  # noqa: SLF001
        saved = [p.out for p in passes], s.loss_out
        try:
            for k, (h, o, b) in enumerate(zip(self.handles, self.offs[:-1], self.sizes)):
                for p in passes:
                    p.out = self.out[o : o + b].data_ptr()
                s.loss_out = self.loss[k : k + 1]
                s.step(h, global_batch=b)
        finally:
            for p, v in zip(passes, saved[0]):
                p.out = v
            s.loss_out = saved[1]

    def _load(self, order):
        self.pin.copy_(torch.from_numpy(np.asarray(order, dtype=np.int64)))
        self.gids.copy_(self.pin, non_blocking=True)
        torch.index_select(self.table, 0, self.gids, out=self.descs)

    def run(self, batches):
        """Train on ``batches`` (lists of dataset positions = graph ids of the
        store, sizes as built); returns (per-batch losses [nb], predictions
        [n, out]) as device tensors, in batch order."""
        if [len(b) for b in batches] != self.sizes:
            msg = "epoch batches do not match the runner's batch sizes"
            raise ValueError(msg)
        self._load(np.concatenate([np.asarray(b) for b in batches]) if batches else [])
        s = self.step
        if self.graph is None:
            # the first use: eager warm-up steps (LDS attributes, the allocator),
            # the capture, the training state put back, then the real replay
            s._packed()  # noqa: SLF001
            snap = [t.detach().clone() for t in s._state_tensors()]  # noqa: SLF001
            n0 = s.step_count
            self._steps()
            torch.cuda.synchronize(s.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._steps()
            torch.cuda.synchronize(s.device)
            for t, v in zip(s._state_tensors(), snap):  # noqa: SLF001
                t.data.copy_(v)
            s.step_count = n0
            self.graph = g
        self.graph.replay()
        s.step_count += len(self.sizes)
        return self.loss, self.out


def runner_for(step, store, sizes, cache: dict):
    """The cached EpochRunner of (step, store, batch sizes), or None when not eligible."""
    key = (id(step), id(store), tuple(int(s) for s in sizes))
    r = cache.get(key)
    if r is None:
        if not (_lib.load() and eligible(step, store)):
            return None
        r = EpochRunner(step, store, sizes)
        cache.clear()  # one runner at a time (its graph holds the step's buffers)
        cache[key] = r
    return r
