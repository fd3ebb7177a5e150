"""Diagnostic: in-graph cost of each launch of a GINet training step.

Captures sweeps (16 resident mini-batches) of (a) full steps, (b) the graph
pass alone, (c) the reduce+Adam alone, and times their replays, so the
per-step share of each launch is measured where it runs (inside a hipGraph,
reading the data the previous launch just wrote)."""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deeprank-gnn-2_amd")]

from bench import make_graphs, records  # noqa: E402
from deeprank2_amd import _lib  # noqa: E402
from deeprank2_amd.engine import FusedTrainStep  # noqa: E402
from deeprank2_amd.fused import BatchHandle, launch  # noqa: E402
from deeprank2_amd.neuralnets.gnn.ginet import GINet  # noqa: E402
from deeprank2_amd.store import GraphStore, pack_graphs  # noqa: E402


def replay_us(g, steps, reps=20):
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / (reps * steps)


def main():
    dev = torch.device("cuda:0")
    nb, B = 16, 64
    packed = pack_graphs(records(make_graphs("residue", nb * B, 1000)))
    store = GraphStore(packed, dev)
    hs = [BatchHandle(store, np.arange(i * B, (i + 1) * B, dtype=np.int32)) for i in range(nb)]
    torch.manual_seed(0)
    step = FusedTrainStep(GINet(30, 1, 3).to(dev).train())
    for h in hs:
        step.step(h)
    torch.cuda.synchronize()
    lib = _lib.load()
    stream = lambda: _lib.stream_ptr(dev)  # noqa: E731

    def cap(body):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for h in hs:
                body(h)
        return g

    def graph_only(h):
        p = step._pass  # noqa: SLF001
        p.loss_scale = 1.0 / B
        launch(step.spec, h, step._w, p)  # noqa: SLF001

    def reduce_only(h):
        _lib.check(lib.dr_reduce_update(step._table, step.slab.data_ptr(), step.head.data_ptr(), h.B, step._adam, step.lpg.data_ptr(), 1.0 / B, step.loss_out.data_ptr(), stream()), "reduce")  # noqa: SLF001

    def reduce_noadam(h):
        _lib.check(lib.dr_reduce_update(step._table, step.slab.data_ptr(), step.head.data_ptr(), h.B, step._adam_off, step.lpg.data_ptr(), 1.0 / B, step.loss_out.data_ptr(), stream()), "reduce")  # noqa: SLF001

    def reduce_b8(h):
        _lib.check(lib.dr_reduce_update(step._table, step.slab.data_ptr(), step.head.data_ptr(), 8, step._adam_off, None, 1.0, None, stream()), "reduce")  # noqa: SLF001

    full = step.capture_sweep(hs)
    r_noadam = cap(reduce_noadam)
    r_b8 = cap(reduce_b8)
    g_only = cap(graph_only)
    r_only = cap(reduce_only)
    print(f"full step          : {replay_us(full, nb):7.2f} us/step")
    print(f"graph pass only    : {replay_us(g_only, nb):7.2f} us/step")
    print(f"reduce+Adam only   : {replay_us(r_only, nb):7.2f} us/step")
    print(f"reduce, no Adam    : {replay_us(r_noadam, nb):7.2f} us/step")
    print(f"reduce B=8 no Adam : {replay_us(r_b8, nb):7.2f} us/step")


if __name__ == "__main__":
    main()
