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
steps (``tests/test_gpu_trainer.py``).  Eligible: fp32, the model's per-graph
kernel holding every graph of the dataset, no non-finite inputs, MSE or
unweighted cross-entropy (the loss scale then depends only on the batch size).

Data parallel (``Trainer(ngpu>1)``, one process per GPU over RCCL): each rank
captures ITS shards of the epoch's global batches — graph pass, gradient
reduce, the RCCL all-reduce of the flat gradient buffer and Adam per step,
the all-reduce inside the graph (as ``bench.py --gpus N`` replays it) — with
each step's local loss term written into the epoch's loss vector; the loss
vector is summed over the ranks once per epoch and the predictions are
gathered once per epoch (``Trainer._epoch_captured``).  RCCL only (a gloo
collective is not a device operation a HIP graph can hold), and every rank's
shard of every batch non-empty.

``EvalRunner``: the forward passes of an evaluation (``Trainer._eval``,
reference ``trainer.py:726-794``) over a loader's batches as one HIP graph,
each pass writing its predictions into an epoch buffer; the per-batch losses
are then the same torch calls on slices of that buffer.
"""

from __future__ import annotations

import numpy as np
import torch

from deeprank2_amd import _lib
from deeprank2_amd.fused import LDS_MAX, BatchHandle, lds_for


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
    h.force_large = h.force_layers = False
    h.large_tile = h.vanilla_split = h.fault = None
    h.large_halos = h.large_atomic_max = h.vanilla_words = True
    h.vanilla_tile_rows = 0
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
    if step.compute_dtype != "f32" or spec.run is not None:
        return False
    if step.pg is not None and (torch.distributed.get_backend(step.pg) != "nccl" or step.device_div):
        return False
    if step.loss == "ce" and step.class_weights is not None:
        return False
    nf = store.packed.nonfinite
    if nf is not None and bool(np.asarray(nf).any()):
        return False
    probe = _static_handle(store, None, 1, store.max_sizes(np.arange(store.packed.n_graphs)))
    return lds_for(spec, probe, step.out_dim) <= LDS_MAX


class EpochRunner:
    """The fused steps of one epoch's batches (sizes ``sizes``, in order) as one HIP graph."""

    def __init__(self, step, store, sizes, global_sizes=None):
        self.step, self.store = step, store
        self.sizes = [int(s) for s in sizes]
        # the loss scale of a data-parallel step is 1/(global batch)
        self.global_sizes = self.sizes if global_sizes is None else [int(s) for s in global_sizes]
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
                s.step(h, global_batch=self.global_sizes[k])
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
            if s.pg is not None:
                # the loss terms go to the epoch's loss vector (summed over the
                # ranks once per epoch): the flat buffer's loss slot, all-reduced
                # with the gradients every step, stays zero
                s.loss_out.zero_()
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


def runner_for(step, store, sizes, cache: dict, global_sizes=None):
    """The cached EpochRunner of (step, store, batch sizes), or None when not eligible."""
    key = (id(step), id(store), tuple(int(s) for s in sizes), None if global_sizes is None else tuple(int(s) for s in global_sizes))
    r = cache.get(key)
    if r is None:
        if not (_lib.load() and eligible(step, store)) or any(int(s) < 1 for s in sizes):
            return None
        r = EpochRunner(step, store, sizes, global_sizes)
        for k in [k for k in cache if not isinstance(k, tuple) or k[0] != "eval"]:
            del cache[k]  # one training runner at a time (its graph holds the step's buffers)
        cache[key] = r
    return r


class EvalRunner:
    """Forward passes (no dropout, no backward) of one evaluation's batches
    (sizes ``sizes``, in order) as one HIP graph; returns the predictions
    [n, out] in batch order.  The same launch as ``model(batch)`` in eval
    mode (``FusedFn.forward``: ``dr_*_graph_pass`` with DR_PASS_FORWARD), so
    the predictions are bit-identical to the per-batch loop's."""

    def __init__(self, model, store, sizes):
        self.model, self.store = model, store
        self.spec = model.fused_spec
        self.sizes = [int(s) for s in sizes]
        self.offs = np.concatenate([[0], np.cumsum(self.sizes)]).astype(np.int64)
        n, dev = int(self.offs[-1]), store.device
        self.out_dim = model.output_shape
        self.table = descriptor_table(store)
        self.pin = torch.empty(n, dtype=torch.int64, pin_memory=True)
        self.gids = torch.empty(n, dtype=torch.int64, device=dev)
        self.descs = torch.empty(n, 64, dtype=torch.uint8, device=dev)
        ms = store.max_sizes(np.arange(store.packed.n_graphs))
        self.handles = [_static_handle(store, self.descs[o : o + b].view(-1), b, ms) for o, b in zip(self.offs[:-1], self.sizes)]
        self.out = torch.empty(n, self.out_dim, dtype=torch.float32, device=dev)
        self.params = model.ordered_params()
        self.w = self.spec.weights(self.params)  # device pointers: Adam updates the parameters in place
        self.graph = None

    def _passes(self):
        from deeprank2_amd.fused import launch, make_pass  # noqa: PLC0415

        for h, o, b in zip(self.handles, self.offs[:-1], self.sizes):
            launch(self.spec, h, self.w, make_pass(self.out_dim, _lib.DR_PASS_FORWARD, out=self.out[o : o + b]))

    def run(self, batches):
        if [len(b) for b in batches] != self.sizes:
            msg = "evaluation batches do not match the runner's batch sizes"
            raise ValueError(msg)
        self.pin.copy_(torch.from_numpy(np.concatenate([np.asarray(b) for b in batches]).astype(np.int64)))
        self.gids.copy_(self.pin, non_blocking=True)
        torch.index_select(self.table, 0, self.gids, out=self.descs)
        if self.graph is None:
            self._passes()  # warm-up (LDS attributes, the allocator); a forward changes no state
            torch.cuda.synchronize(self.store.device)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g):
                self._passes()
            self.graph = g
        self.graph.replay()
        return self.out


def eval_eligible(model, store) -> bool:
    spec = getattr(model, "fused_spec", None)
    if spec is None or spec.run is not None or model.training:
        return False
    nf = store.packed.nonfinite
    if nf is not None and bool(np.asarray(nf).any()):
        return False
    probe = _static_handle(store, None, 1, store.max_sizes(np.arange(store.packed.n_graphs)))
    return lds_for(spec, probe, model.output_shape) <= LDS_MAX


def eval_runner_for(model, store, sizes, cache: dict):
    """The cached EvalRunner of (model, store, batch sizes), or None when not eligible."""
    key = ("eval", id(model), id(store), tuple(int(s) for s in sizes))
    r = cache.get(key)
    if r is None:
        if not sizes or any(int(s) < 1 for s in sizes) or not (_lib.load() and eval_eligible(model, store)):
            return None
        r = EvalRunner(model, store, sizes)
        cache[key] = r
    return r
