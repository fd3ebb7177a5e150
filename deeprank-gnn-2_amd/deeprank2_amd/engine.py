"""Fused GINet training step: the hot loop of ``Trainer._epoch``
(reference ``deeprank2/trainer.py:682-690``) in two launches per mini-batch.

1. ``dr_ginet_graph_pass`` (FORWARD|BACKWARD, loss in-kernel): one workgroup
   per graph computes the prediction, the loss term and the whole backward of
   its graph, writing per-graph partials;
2. ``dr_ginet_reduce_update``: sums the partials into the 16 gradients and
   applies ``torch.optim.Adam`` (lr, betas, eps, L2 ``weight_decay`` as
   ``Trainer.configure_optimizers`` sets them, trainer.py:401-428).

Data parallel (one process per GPU, RCCL over xGMI): every rank runs step 1 on
its shard of the global batch with the loss scaled by 1/B_global, the 16
gradients (one flat 42.7 KB buffer for GINet(30,1,3)) are SUM-all-reduced, then
step 2 runs Adam from the reduced gradients.  That is the only collective.
"""

from __future__ import annotations

import math

import torch

from deeprank2_amd import _lib
from deeprank2_amd.neuralnets.gnn.ginet import BatchHandle, Dropout, GINet, graph_pass, head_stride, reduce_update, slab_stride


class GINetTrainStep:
    def __init__(self, model: GINet, lr=1e-3, weight_decay=1e-5, betas=(0.9, 0.999), eps=1e-8, loss="mse", class_weights=None, process_group=None):
        self.model = model
        self.params = model.ordered_params()
        for p in self.params:
            if not p.is_cuda or not p.is_contiguous() or p.dtype != torch.float32:
                msg = "GINetTrainStep needs contiguous fp32 cuda parameters"
                raise ValueError(msg)
        dev = self.params[0].device
        self.device = dev
        self.out_dim = model.output_shape
        self.lr, self.weight_decay, self.betas, self.eps = lr, weight_decay, betas, eps
        self.loss = loss
        self.class_weights = None if class_weights is None else torch.as_tensor(class_weights, dtype=torch.float32, device=dev)
        self.pg = process_group
        self.world = torch.distributed.get_world_size(process_group) if process_group is not None else 1
        numel = [p.numel() for p in self.params]
        self.flat_grad = torch.zeros(sum(numel), dtype=torch.float32, device=dev)
        self.grads = list(torch.split(self.flat_grad, numel))
        self.grads = [g.view_as(p) for g, p in zip(self.grads, self.params)]
        self.states = [(torch.zeros_like(p), torch.zeros_like(p)) for p in self.params]
        self.step_count = 0
        self.loss_out = torch.zeros(1, dtype=torch.float32, device=dev)
        self.kernel_events = None  # list -> (start, end) HIP events around each graph pass
        self._cap = 0
        self._ensure(64)

    def _ensure(self, b):
        if b <= self._cap:
            return
        f = self.model.input_shape
        dev = self.device
        self.slab = torch.empty(b * slab_stride(f), dtype=torch.float32, device=dev)
        self.head = torch.empty(b * head_stride(self.out_dim), dtype=torch.float32, device=dev)
        self.lpg = torch.empty(b, dtype=torch.float32, device=dev)
        self.out = torch.empty(b, self.out_dim, dtype=torch.float32, device=dev)
        self._cap = b

    def loss_scale(self, h: BatchHandle, global_batch):
        if self.loss == "mse":
            return 1.0 / (global_batch * self.out_dim if self.out_dim > 1 else global_batch)
        if self.class_weights is None:
            return 1.0 / global_batch
        y = h.store.packed.y[h.gids_host].astype(int)
        wsum = float(self.class_weights.cpu().numpy()[y].sum())
        if self.world > 1:
            t = torch.tensor([wsum], dtype=torch.float64)
            torch.distributed.all_reduce(t, group=self.pg)
            wsum = float(t.item())
        return 1.0 / wsum

    def adam_c(self, enabled=True):
        a = _lib.AdamC()
        t = self.step_count
        a.lr, (a.beta1, a.beta2), a.eps, a.weight_decay = self.lr, self.betas, self.eps, self.weight_decay
        a.bias_c1 = 1.0 - self.betas[0] ** t
        a.bias_c2_sqrt = math.sqrt(1.0 - self.betas[1] ** t)
        a.enabled = int(enabled)
        return a

    def step(self, h: BatchHandle, mask=None, global_batch=None, dropout=True):
        """One training step on the graphs of ``h``; returns (loss [1], out [B,out]) device views.

        Dropout (ginet.py:122): ``mask`` (uint8 [B,128]) if given, else the
        in-kernel hash RNG when ``dropout`` and the model's p > 0."""
        self._ensure(h.B)
        if global_batch is None:
            global_batch = h.B * self.world
        kind = _lib.DR_LOSS_MSE if self.loss == "mse" else _lib.DR_LOSS_CE
        scale = self.loss_scale(h, global_batch)
        drop = None
        if mask is not None:
            drop = Dropout(self.model.dropout, mask=mask)
        elif dropout and self.model.dropout > 0:
            drop = self.model.next_dropout()
        ev = self.kernel_events
        if ev is not None:
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
        graph_pass(
            h, self.params, self.out_dim, _lib.DR_PASS_FORWARD | _lib.DR_PASS_BACKWARD,
            dropout=drop, loss_kind=kind, loss_scale=scale, class_w=self.class_weights,
            out=self.out, loss_per_graph=self.lpg, slab=self.slab, head=self.head,
        )  # fmt: skip
        if ev is not None:
            e1.record()
            ev.append((e0, e1))
        self.step_count += 1
        if self.world == 1:
            reduce_update(h, self.params, self.grads, self.out_dim, self.slab, self.head, adam=self.adam_c(), states=self.states, loss_per_graph=self.lpg, loss_scale=scale, loss_out=self.loss_out)
        else:
            reduce_update(h, self.params, self.grads, self.out_dim, self.slab, self.head, adam=self.adam_c(False), loss_per_graph=self.lpg, loss_scale=scale, loss_out=self.loss_out)
            torch.distributed.all_reduce(self.flat_grad, group=self.pg)
            torch.distributed.all_reduce(self.loss_out, group=self.pg)
            reduce_update(h, self.params, self.grads, self.out_dim, None, None, adam=self.adam_c(), states=self.states)
        return self.loss_out, self.out[: h.B]
