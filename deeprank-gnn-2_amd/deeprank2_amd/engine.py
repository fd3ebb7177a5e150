"""Fused training step: the hot loop of ``Trainer._epoch``
(reference ``deeprank2/trainer.py:682-690``) in two launches per mini-batch,
for any model with a ``fused_spec`` (GINet, FoutNet).

1. the model's graph pass (``dr_ginet_graph_pass`` / ``dr_fout_graph_pass``;
   FORWARD|BACKWARD, loss in-kernel): one workgroup per graph computes the
   prediction, the loss term and the whole backward of its graph, writing
   per-graph partials;
2. ``dr_reduce_update``: sums the partials into every gradient and
   applies ``torch.optim.Adam`` (lr, betas, eps, L2 ``weight_decay`` as
   ``Trainer.configure_optimizers`` sets them, trainer.py:401-428).

The dropout offset and Adam's step number live in a device counter that the
two kernels advance themselves, so a step's launch arguments are constant and
the whole step can be captured once per mini-batch and replayed as a HIP graph
(``capture``).

Data parallel (one process per GPU, RCCL over xGMI): every rank runs step 1 on
its shard of the global batch with the loss scaled by 1/B_global, the
gradients and the loss term (one flat buffer: 42.7 KB for GINet(30,1,3),
16.8 KB for FoutNet(30,1)) are SUM-all-reduced, then step 2 runs Adam from the
reduced gradients.  That is the only collective (``distributed.py`` shards).
"""

from __future__ import annotations

import ctypes

import torch

from deeprank2_amd import _lib, layered
from deeprank2_amd.fused import BatchHandle, launch, param_table, slab_rows_for


class FusedTrainStep:
    # the accumulating pass's defaults for new step objects (instance
    # attributes acc / acc_groups override them; tests set these to drive the
    # Trainer's own steps)
    acc_default = None
    acc_groups_default = None

    def __init__(self, model, lr=1e-3, weight_decay=1e-5, betas=(0.9, 0.999), eps=1e-8, loss="mse", class_weights=None, process_group=None, max_batch=64, compute_dtype="f32"):
        self.model = model
        if compute_dtype not in ("f32", "bf16"):
            msg = f"compute_dtype must be 'f32' or 'bf16' (got {compute_dtype!r})"
            raise ValueError(msg)
        if compute_dtype == "bf16" and not getattr(model.fused_spec, "bf16", False):
            msg = f"{type(model).__name__} has no bf16 compute path (GINet has: BASELINE.json configs[3])"
            raise ValueError(msg)
        self.compute_dtype = compute_dtype
        self.spec = model.fused_spec
        self.params = model.ordered_params()
        for p in self.params:
            if not p.is_cuda or not p.is_contiguous() or p.dtype != torch.float32:
                msg = "FusedTrainStep needs contiguous fp32 cuda parameters"
                raise ValueError(msg)
        dev = self.params[0].device
        self.device = dev
        self.out_dim = model.output_shape
        self.lr, self.weight_decay, self.betas, self.eps = lr, weight_decay, betas, eps
        if loss not in ("mse", "ce"):
            msg = f"loss must be 'mse' or 'ce' (got {loss!r})"
            raise ValueError(msg)
        self.loss = loss
        self.class_weights = None if class_weights is None else torch.as_tensor(class_weights, dtype=torch.float32, device=dev)
        # host copy, taken once: the per-batch weight sum never syncs with the device
        self._cw_host = None if class_weights is None else torch.as_tensor(class_weights, dtype=torch.float32).detach().cpu().numpy()
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        numel = [p.numel() for p in self.params]
        # gradients, the loss and (weighted CE, N>1) the batch's class-weight sum
        # share one buffer: one all-reduce per step (N>1)
        # (models whose graph pass has in-launch hand-offs: + the pass's fault flag,
        # so a give-up on any rank withholds the update on every rank)
        self.handoffs = bool(getattr(self.spec, "handoffs", False))
        extra = 3 if self.handoffs else 2
        self.flat = torch.zeros(sum(numel) + extra, dtype=torch.float32, device=dev)
        self.flat_grad = self.flat[: sum(numel)]
        self.grads = [g.view_as(p) for g, p in zip(torch.split(self.flat_grad, numel), self.params)]
        self.states = [(torch.zeros_like(p), torch.zeros_like(p)) for p in self.params]
        self.counter = torch.zeros(2, dtype=torch.int64, device=dev)  # [steps done = dropout offset, snapshot]
        self.step_count = 0
        self.loss_out = self.flat[sum(numel) : sum(numel) + 1]
        self.wsum = self.flat[sum(numel) + 1 : sum(numel) + 2]
        self.flat_fault = self.flat[sum(numel) + 2 :]  # (handoffs) fault[0] of this rank, summed over ranks
        # dr_pass.fault: [0] = this step's graph pass gave up a hand-off (cleared
        # by every launch), [1] = such launches since the last check_faults();
        # fault_red: [0] after the all-reduce (N>1)
        self.fault = torch.zeros(2, dtype=torch.int32, device=dev)
        self.fault_red = torch.zeros(1, dtype=torch.int32, device=dev)
        # weighted CE with N>1: the graph pass runs unnormalised and Adam divides
        # by the all-reduced weight sum (dr_adam.grad_div)
        self.device_div = self.loss == "ce" and self.class_weights is not None and self.world > 1
        self.kernel_events = None  # list -> (start, end) HIP events around each graph pass
        # (r03-r05 also shipped one-launch, reduce-at-start and pipelined GINet
        # steps and a sibling split of the per-graph kernel; all measured slower
        # than these two launches and removed in r06)
        # accumulating pass (GINet fp32, batches past the CU count;
        # dr_ginet_acc_pass): acc_groups workgroups each run every
        # acc_groups-th graph and sum the gradients on chip, one row each,
        # so the reduce reads acc_groups rows instead of B per-graph partials.
        # None = auto (B > the device's CU count), False = off, True = on
        # wherever the batch allows it.  Another fp32 association than the
        # per-graph partials (deterministic).
        self.acc = self.acc_default
        self.acc_groups = self.acc_groups_default  # workgroups (None: the CU count)
        self._acc_slab = None
        self._table_acc = None
        self._cus = None  # the device's CU count (queried once)
        # models whose graph pass reads its weights from a packed copy
        # (VanillaNetwork: MFMA-fragment order): one copy per step object,
        # rewritten by Adam as it updates the parameters (dr_adam.mirror), so
        # the pass needs no pack launch (DR_PASS_WPACK_CURRENT); repacked when
        # the parameters change outside the step (torch's version counters).
        # The Adam call that follows such a pass also clears its fault flag
        # (dr_adam.fault_clear), which the pack launch used to do.
        self.wpack = None  # (buffer, mirror_idx, refresh), made on first use
        self._wpack_ver = None
        self.ticket = torch.zeros(1, dtype=torch.int32, device=dev)
        if getattr(model, "_drop_seed", 0) is None:
            model._drop_seed = int(torch.randint(0, 2**62, (1,)).item())
        self._cap = 0
        self._ensure(max_batch)

    # ---- persistent C structs (built once; a step makes two ctypes calls) ----
    def _ensure(self, b):
        if b <= self._cap:
            return
        f = self.model.input_shape
        dev = self.device
        self.slab = torch.empty(b * self.spec.slab_stride(f), dtype=torch.float32, device=dev)
        self.head = torch.zeros(b * self.spec.head_stride(self.out_dim), dtype=torch.float32, device=dev)
        self.lpg = torch.empty(b, dtype=torch.float32, device=dev)
        self.out = torch.empty(b, self.out_dim, dtype=torch.float32, device=dev)
        self._cap = b
        self._build_structs()

    def _build_structs(self):
        p = _lib.PassC()
        p.flags = _lib.DR_PASS_FORWARD | _lib.DR_PASS_BACKWARD
        p.out_dim = self.out_dim
        p.loss_kind = _lib.DR_LOSS_MSE if self.loss == "mse" else _lib.DR_LOSS_CE
        if self.spec.dropout > 0 and self.model.dropout > 0:
            p.use_dropout = _lib.DR_DROPOUT_HASH
            p.drop_p = self.model.dropout
            p.drop_scale = 1.0 / (1.0 - self.model.dropout)
            p.drop_seed = self.model._drop_seed
        p.class_w = _lib.ptr(self.class_weights)
        p.out = self.out.data_ptr()
        p.loss_per_graph = self.lpg.data_ptr()
        p.slab = self.slab.data_ptr()
        p.head = self.head.data_ptr()
        p.step_counter = self.counter.data_ptr()
        p.compute_dtype = _lib.DR_DTYPE_BF16 if self.compute_dtype == "bf16" else _lib.DR_DTYPE_F32
        p.fault = self.fault.data_ptr()
        self._pass = p
        self._pass_nodrop = _lib.PassC.from_buffer_copy(p)
        self._pass_nodrop.use_dropout = _lib.DR_DROPOUT_OFF
        self._w = self.spec.weights(self.params)
        self._table = param_table(self.spec, self.params, self.grads, self.states, self.model.input_shape, self.out_dim)
        a = _lib.AdamC()
        a.lr, (a.beta1, a.beta2), a.eps, a.weight_decay = self.lr, self.betas, self.eps, self.weight_decay
        a.enabled = 1
        a.step_counter = self.counter.data_ptr()
        # world of one: this step's own flag; N>1: the all-reduced one (the
        # partial reduce before the all-reduce NaNs the rank's gradients)
        a.fault = (self.fault if self.pg is None else self.fault_red).data_ptr()
        self._adam = a
        self._adam_off = _lib.AdamC.from_buffer_copy(a)
        self._adam_off.enabled = 0
        self._adam_off.fault = self.fault.data_ptr()
        self._adam_div = _lib.AdamC.from_buffer_copy(a)
        self._adam_div.grad_div = self.wsum.data_ptr()
        self._table_acc = None  # rebuilt on first use (parameters / grads may have moved)
        self._wire_packed()

    def _wire_packed(self):
        """The updating Adam calls (not the gradients-only one before an
        all-reduce) rewrite the packed copy and clear the pass's fault flag
        (N>1: after the flag was copied into the all-reduced buffer)."""
        if self.wpack is None:
            return
        for a in (self._adam, self._adam_div):
            a.mirror, a.mirror_idx = self.wpack[0].data_ptr(), self.wpack[1].data_ptr()
            a.fault_clear, a.ticket = self.fault.data_ptr(), self.ticket.data_ptr()

    packed_mirror = True  # False: the pass packs the weights itself every launch (A/B switch)

    def _packed(self):
        """The packed weight copy, current for the parameters as they are now
        (None: the model has none, or ``packed_mirror`` is off)."""
        if not self.packed_mirror or getattr(self.spec, "wpack", None) is None:
            return None
        ver = tuple(p._version for p in self.params)
        if self.wpack is None:
            self.wpack = self.spec.wpack(self.params)
            self._wpack_ver = ver
            self._wire_packed()
        elif ver != self._wpack_ver:  # changed outside the step (load_state_dict, an optimizer, ...)
            self.wpack[2]()
            self._wpack_ver = ver
        return self.wpack[0]

    def refresh_packed(self):
        """Repack the model's packed weight copy from the parameters now."""
        if self.wpack is not None:
            self.wpack[2]()
            self._wpack_ver = tuple(p._version for p in self.params)

    def loss_scale(self, h: BatchHandle, global_batch):
        """Factor of the per-graph loss terms: 1/B (MSE: 1/(B*out)), or for a
        weighted CrossEntropyLoss 1/sum_b w[y_b] — computed on the host from the
        stored targets.  With N>1 that sum spans all ranks: the pass then runs
        with factor 1, the local sum goes into the all-reduced buffer and Adam
        divides by the reduced one (``device_div``)."""
        if self.loss == "mse":
            return 1.0 / (global_batch * self.out_dim if self.out_dim > 1 else global_batch)
        if self.class_weights is None:
            return 1.0 / global_batch
        if self.device_div:
            return 1.0
        y = h.store.packed.y[h.gids_host].astype(int)
        return 1.0 / float(self._cw_host[y].sum())

    def _local_wsum(self, h: BatchHandle):
        y = h.store.packed.y[h.gids_host].astype(int)
        self.wsum.fill_(float(self._cw_host[y].sum()))

    def _adam_after_allreduce(self):
        lib = _lib.load()
        stream = _lib.stream_ptr(self.device)
        if self.device_div:
            _lib.check(lib.dr_reduce_update(self._table, None, None, 0, self._adam_div, None, 1.0, self.loss_out.data_ptr(), stream), "dr_reduce_update")
        else:
            _lib.check(lib.dr_reduce_update(self._table, None, None, 0, self._adam, None, 1.0, None, stream), "dr_reduce_update")

    def step(self, h: BatchHandle, mask=None, global_batch=None, dropout=True):
        """One training step on the graphs of ``h``; returns (loss [1], out [B,out]) device views.

        Dropout (ginet.py:122): ``mask`` (uint8 [B,128]) if given, else the
        in-kernel hash RNG (offset = the device step counter) when ``dropout``
        and the model's p > 0."""
        self._ensure(h.B)
        if global_batch is None:
            global_batch = h.B * self.world
        scale = self.loss_scale(h, global_batch)
        if self.spec.layers is not None and layered.needs_layers(self.spec, h, self.out_dim):
            return self._layered_step(h, scale, dropout, mask)
        lib = _lib.load()
        stream = _lib.stream_ptr(self.device)
        if mask is not None:
            p = _lib.PassC.from_buffer_copy(self._pass)
            p.use_dropout = _lib.DR_DROPOUT_MASK
            p.drop_scale = 1.0 / (1.0 - self.model.dropout)
            p.mask = mask.data_ptr()
        else:
            p = self._pass if (dropout and self.spec.dropout > 0 and self.model.dropout > 0) else self._pass_nodrop
        p.loss_scale = scale
        ev = self.kernel_events
        if ev is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        rows = self._launch_pass(h, p)
        if ev is not None:
            e1.record()
            ev.append((e0, e1))
        self.step_count += 1
        table, slab, n_rows = self._reduce_args(h, rows)
        head, lpg, lout = self.head.data_ptr(), self.lpg.data_ptr(), self.loss_out.data_ptr()
        if self.pg is None:
            _lib.check(lib.dr_reduce_update(table, slab, head, n_rows, self._adam, lpg, scale, lout, stream), "dr_reduce_update")
        else:
            _lib.check(lib.dr_reduce_update(table, slab, head, n_rows, self._adam_off, lpg, scale, lout, stream), "dr_reduce_update")
            if self.device_div:
                self._local_wsum(h)
            if self.handoffs:
                self.flat_fault.copy_(self.fault[:1])
            torch.distributed.all_reduce(self.flat, group=self.pg)
            if self.handoffs:
                self.fault_red.copy_(self.flat_fault)
            self._adam_after_allreduce()
        return self.loss_out, self.out[: h.B]

    def _acc_rows(self, h: BatchHandle) -> int:
        """Workgroups (= partial rows) of the accumulating pass for this
        batch, or 0 when the batch takes the per-graph partials."""
        from deeprank2_amd.fused import _device_cus, lds_for  # noqa: PLC0415

        if self.acc is False or self.spec.entry != "dr_ginet_graph_pass" or self.compute_dtype != "f32":
            return 0
        if h.nonfinite or h.force_large or self.spec.layers is not None and layered.needs_layers(self.spec, h, self.out_dim):
            return 0
        if self._cus is None:
            self._cus = _device_cus(self.device)
        r = int(self.acc_groups or self._cus)
        if self.acc is None and h.B <= r:
            return 0
        f = self.model.input_shape
        lib = _lib.load()
        if self.acc_lds(h) > 160 * 1024:  # noqa: PLR2004
            return 0
        r = min(r, h.B)
        rs = int(lib.dr_ginet_acc_row_floats(f, self.out_dim))
        if self._acc_slab is None or self._acc_slab.numel() < r * rs:
            self._acc_slab = torch.empty(r * rs, dtype=torch.float32, device=self.device)
        if self._table_acc is None:
            from deeprank2_amd.fused import param_table  # noqa: PLC0415

            self._table_acc = param_table(self.spec, self.params, self.grads, self.states, f, self.out_dim)
            slab, z = _lib.DR_GRAD_SLAB, (_lib.DR_GRAD_ZERO, 0, 0, 0)
            c0 = 32 * f + 1024
            rec = [
                (slab, 0, 0, 0), z, z, (slab, 32 * f, 0, 0), z, z,
                (slab, 16 * f, 0, 0), z, z, (slab, 32 * f + 512, 0, 0), z, z,
                (slab, c0, 0, 0), (slab, c0 + 8192, 0, 0), (slab, c0 + 8320, 0, 0), (slab, c0 + 8320 + 128 * self.out_dim, 0, 0),
            ]  # fmt: skip
            for i, (kind, o1, o2, cols) in enumerate(rec):
                t = self._table_acc.recipe[i]
                t.kind, t.off1, t.off2, t.cols = kind, o1, o2, cols
            self._table_acc.slab_stride = rs
            self._table_acc.slab_rows = 1
        return r

    # the accumulating pass's prefetch layout where it fits: the next graph's
    # inputs staged by the waves with no tile in the front half (DESIGN §5;
    # B = 4096: 233.7 -> 224.3 us/step)
    acc_prefetch = True

    def _acc_max_sizes(self, h: BatchHandle):
        if not self.acc_prefetch:
            return None
        key = "acc_max_sizes"
        m = h._lds.get(key)  # noqa: SLF001
        if m is None:
            m = h._lds[key] = (ctypes.c_int32 * 5)(*h.max_sizes)  # noqa: SLF001
        return m

    def acc_lds(self, h: BatchHandle) -> int:
        """Dynamic LDS bytes the accumulating pass takes for this batch: the
        prefetch layout when it fits, else the largest graph's carve plus the
        accumulators."""
        from deeprank2_amd.fused import lds_for  # noqa: PLC0415

        f, out = self.model.input_shape, self.out_dim
        m = self._acc_max_sizes(h)
        if m is not None:
            pf = int(_lib.load().dr_ginet_acc_lds_bytes(m, f, int(h.store.packed.transpose_aliased), out))
            if 0 < pf <= 160 * 1024:  # noqa: PLR2004
                return pf
        words = 32 * f + 1024 + ((128 + 128 * out + out + 1 + 3) & ~3) + (8192 if f > 32 else 0) + 4  # noqa: PLR2004
        return lds_for(self.spec, h, out) + 4 * words

    def _launch_pass(self, h: BatchHandle, p) -> int:
        """The graph pass of a two-launch step: the accumulating pass (returns
        its row count) or the model's per-graph pass (returns 0)."""
        from deeprank2_amd.fused import lds_for  # noqa: PLC0415

        r = self._acc_rows(h)
        if r == 0:
            launch(self.spec, h, self._w, p, wpack=self._packed())
            return 0
        p.slab = self._acc_slab.data_ptr()
        try:  # (no plan: workgroup w runs positions w, w + r, ... — the same order eager and captured)
            rc = _lib.load().dr_ginet_acc_pass(h.store.cstruct(), h.descs.data_ptr(), h.B, self._w, p, lds_for(self.spec, h, self.out_dim), r, None, self._acc_max_sizes(h), _lib.stream_ptr(self.device))
        finally:
            p.slab = self.slab.data_ptr()
        _lib.check(rc, "dr_ginet_acc_pass")
        return r

    def _reduce_args(self, h: BatchHandle, acc_rows: int):
        """(table, slab pointer, rows) of the reduce after a pass that
        returned ``acc_rows`` from :meth:`_launch_pass`."""
        if acc_rows:
            return self._table_acc, self._acc_slab.data_ptr(), acc_rows
        self._table.slab_rows = slab_rows_for(self.spec, h)
        return self._table, self.slab.data_ptr(), h.B

    def step_empty(self):
        """A rank whose shard of the global batch is empty (global batch smaller
        than the world): zero gradients and loss into the all-reduce, then the
        same Adam step as every other rank."""
        if self.pg is None:
            msg = "an empty batch only occurs as a data-parallel shard"
            raise ValueError(msg)
        with torch.no_grad():
            self.flat.zero_()
            self.fault[0].zero_()
            self.counter[1].copy_(self.counter[0])  # the snapshot a graph pass would take
        self.step_count += 1
        torch.distributed.all_reduce(self.flat, group=self.pg)
        if self.handoffs:
            self.fault_red.copy_(self.flat_fault)
        self._adam_after_allreduce()
        return self.loss_out, self.out[:0]

    def check_faults(self, reset=True):
        """Raise RuntimeError if any graph pass since the last check gave up an
        in-launch hand-off (VanillaNetwork split over workgroups whose siblings
        were not co-resident): those steps reported a NaN loss and were not
        applied.  One device read; ``Trainer`` calls it once per epoch.

        With a process group this is a collective (every rank calls it at the
        same point): the per-rank counts are SUM-all-reduced first, so all ranks
        raise together instead of the faulting rank alone while the others
        block in their next collective."""
        if not self.handoffs:
            return
        count = self.fault[1:2].clone()
        if self.pg is not None:
            torch.distributed.all_reduce(count, group=self.pg)
        n = int(count.item())
        if reset:
            self.fault[1].zero_()
        if n:
            msg = (f"{n} graph pass(es) of {type(self.model).__name__} gave up waiting for a sibling workgroup "
                   "(in-launch hand-off timed out): those steps were skipped (NaN loss, no update). "
                   "Run with BatchHandle.vanilla_split = 1, or keep other work off the GPU during training.")
            raise RuntimeError(msg)

    def _layered_step(self, h: BatchHandle, scale, dropout, mask=None):
        """A batch the model's graph pass cannot hold, or (GINet) one with
        non-finite inputs (``layered.py``): the
        layer-level forward (reference forward on the layer kernels), the loss
        of the fused path, autograd gradients into the flat buffer, then the
        same all-reduce (N>1) and Adam kernel as the fused step."""
        t = layered.batch_tensors(h)
        out = self.spec.layers(self.model, t, (dropout or mask is not None) and self.model.training, mask=mask)
        if self.loss == "mse":
            lpg = (out[:, 0] - t.y) ** 2
        else:
            yi = t.y.long()
            lpg = -torch.log_softmax(out, 1).gather(1, yi[:, None])[:, 0]
            if self.class_weights is not None:
                lpg = lpg * self.class_weights[yi]
        loss = lpg.sum() * scale
        grads = torch.autograd.grad(loss, self.params, allow_unused=True)
        with torch.no_grad():
            for g, dst in zip(grads, self.grads):
                if g is None:
                    dst.zero_()
                else:
                    dst.copy_(g)
            self.loss_out.copy_(loss.detach().reshape(1))
            self.out[: h.B].copy_(out.detach())
            self.counter[1].copy_(self.counter[0])  # the step snapshot the graph pass would have taken
        self.step_count += 1
        if self.pg is not None:
            if self.device_div:
                self._local_wsum(h)
            torch.distributed.all_reduce(self.flat, group=self.pg)
        self._adam_after_allreduce()
        return self.loss_out, self.out[: h.B]

    # ---- torch.optim.Adam-compatible optimizer state (checkpoints) ----
    def adam_state_dict(self):
        """The fused optimizer state as ``torch.optim.Adam(model.parameters()).state_dict()``
        would hold it (parameter order = the model's ``parameters()`` order)."""
        opt = torch.optim.Adam(self.params, lr=self.lr, betas=self.betas, eps=self.eps, weight_decay=self.weight_decay)
        t = int(self.counter[0].item())
        if t > 0:
            for p, (m, v) in zip(self.params, self.states):
                opt.state[p] = {"step": torch.tensor(float(t)), "exp_avg": m.detach().clone(), "exp_avg_sq": v.detach().clone()}
        return opt.state_dict()

    def load_adam_state_dict(self, sd):
        """Inverse of :meth:`adam_state_dict` (also accepts a torch Adam state_dict)."""
        group = sd["param_groups"][0]
        if len(group["params"]) != len(self.params) or group.get("amsgrad", False):
            msg = "optimizer state does not match this model (or uses amsgrad)"
            raise ValueError(msg)
        states = sd.get("state", {})
        steps = set()
        for slot, (m, v) in zip(group["params"], self.states):
            st = states.get(slot)
            if st is None:
                m.zero_()
                v.zero_()
                steps.add(0)
                continue
            m.copy_(st["exp_avg"])
            v.copy_(st["exp_avg_sq"])
            steps.add(int(float(st["step"])))
        if len(steps) > 1:
            msg = f"parameters are at different Adam steps {sorted(steps)}"
            raise ValueError(msg)
        t = steps.pop() if steps else 0
        self.counter.fill_(t)
        self.step_count = t
        self.lr, self.betas, self.eps, self.weight_decay = group["lr"], tuple(group["betas"]), group["eps"], group["weight_decay"]
        self._build_structs()

    def _state_tensors(self):
        packed = [] if self.wpack is None else [self.wpack[0]]
        return [*self.params, *[s for st in self.states for s in st], self.counter, self.flat, self.fault, *packed]

    def capture_sweep(self, handles, global_batch=None):
        """Capture one training step per handle, in order, into ONE HIP graph
        (a sweep over the resident mini-batches): replaying it runs
        len(handles) steps with a single graph launch.  Training state is
        left as before the call."""
        for h in handles:
            self._ensure(h.B)
        self._packed()  # made before the snapshot, so the restore covers it
        snap = [t.detach().clone() for t in self._state_tensors()]
        n = self.step_count
        for h in handles:  # warm-up: LDS attributes, plans, allocator
            self.step(h, global_batch=global_batch)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for h in handles:
                self.step(h, global_batch=global_batch)
        torch.cuda.synchronize(self.device)
        for t, s in zip(self._state_tensors(), snap):
            t.data.copy_(s)
        self.step_count = n
        return g

    def time_graph_pass(self, handles, n_launches, global_batch=None):
        """Mean duration (ms) of the model's graph pass alone: ``n_launches``
        passes over ``handles`` (cycled) captured back to back into one HIP
        graph, replayed between two HIP events on the launch stream.  Used for
        ``roofline.achieved``; no host launch overhead enters the number (the
        rocprofv3 kernel average is the cross-check).  State is restored."""
        for h in handles:
            self._ensure(h.B)
        snap = [t.detach().clone() for t in self._state_tensors()]
        n = self.step_count
        p = self._pass if (self.spec.dropout > 0 and self.model.dropout > 0) else self._pass_nodrop

        def passes(k):
            for i in range(k):
                h = handles[i % len(handles)]
                p.loss_scale = self.loss_scale(h, global_batch or h.B * self.world)
                self._launch_pass(h, p)

        passes(len(handles))  # warm-up: LDS attributes, plans
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            passes(n_launches)
        g.replay()  # untimed replay (first replay uploads the graph)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize(self.device)
        ms = e0.elapsed_time(e1) / n_launches
        del g
        for t, s in zip(self._state_tensors(), snap):
            t.data.copy_(s)
        self.step_count = n
        return ms

    def time_reduce(self, handles, n_launches, global_batch=None):
        """Mean duration (ms) of the step's second launch alone
        (``dr_reduce_update``: the fixed-order gradient sums + Adam), timed like
        :meth:`time_graph_pass` (``n_launches`` captured back to back, HIP
        events on the launch stream).  With the graph pass's time it splits a
        step into pass / reduce / the rest (launch gaps, host).  State is
        restored.  None where the step has no separate reduce launch
        (data-parallel step, layer-level batches)."""
        if self.pg is not None or any(self.spec.layers is not None and layered.needs_layers(self.spec, h, self.out_dim) for h in handles):
            return None
        lib = _lib.load()
        for h in handles:
            self._ensure(h.B)
        snap = [t.detach().clone() for t in self._state_tensors()]
        n = self.step_count
        for h in handles:  # one real step each, so the slabs hold a batch's partials
            self.step(h, global_batch=global_batch)
        torch.cuda.synchronize(self.device)

        def reduces(k):
            stream = _lib.stream_ptr(self.device)  # inside the capture: the capturing stream
            for i in range(k):
                h = handles[i % len(handles)]
                table, slab, n_rows = self._reduce_args(h, self._acc_rows(h))
                scale = self.loss_scale(h, global_batch or h.B * self.world)
                _lib.check(lib.dr_reduce_update(table, slab, self.head.data_ptr(), n_rows, self._adam, self.lpg.data_ptr(), scale, self.loss_out.data_ptr(), stream), "dr_reduce_update")

        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            reduces(n_launches)
        g.replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        g.replay()
        e1.record()
        torch.cuda.synchronize(self.device)
        ms = e0.elapsed_time(e1) / n_launches
        del g
        for t, s in zip(self._state_tensors(), snap):
            t.data.copy_(s)
        self.step_count = n
        return ms

    def capture(self, h: BatchHandle, global_batch=None, dropout=True):
        """Capture one training step on ``h`` into a HIP graph (``torch.cuda.CUDAGraph``).

        Replaying it runs the same launches (plus the all-reduce for N>1) with
        no host work; the device counter advances the dropout offset and
        Adam's step on every replay.  (A model with a packed weight copy —
        VanillaNetwork — reads it as the replays' Adam leaves it: parameters
        changed outside the graph between replays need a ``step()`` or
        ``refresh_packed()`` first.)  Capturing does not change the training
        state (the warm-up step it needs is rolled back)."""
        self._ensure(h.B)
        self._packed()  # made before the snapshot, so the restore covers it
        snap = [t.detach().clone() for t in self._state_tensors()]
        n = self.step_count
        self.step(h, global_batch=global_batch, dropout=dropout)  # warm-up: LDS attribute, allocator
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.step(h, global_batch=global_batch, dropout=dropout)
        torch.cuda.synchronize(self.device)
        for t, s in zip(self._state_tensors(), snap):
            t.data.copy_(s)
        self.step_count = n
        return g


GINetTrainStep = FusedTrainStep  # GINet's fused spec drives it
