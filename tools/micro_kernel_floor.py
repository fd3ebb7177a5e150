"""Diagnostic: the floor of a kernel launch on this GPU versus dr_reduce_update.

Times (HIP events, eager, same stream) an empty torch kernel-sized op, the
reduce+Adam kernel alone on resident partials, and graph-pass + reduce pairs,
to separate fixed launch/cache-maintenance cost from the reduction's own work.
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deeprank-gnn-2_amd")]

from bench import records  # noqa: E402
from deeprank2_amd import _lib  # noqa: E402
from deeprank2_amd.engine import FusedTrainStep  # noqa: E402
from deeprank2_amd.fused import BatchHandle  # noqa: E402
from deeprank2_amd.neuralnets.gnn.ginet import GINet  # noqa: E402
from deeprank2_amd.store import GraphStore, pack_graphs  # noqa: E402
from deeprank2_amd.utils.synthetic import make_dataset  # noqa: E402


def timed(fn, n=200):
    for _ in range(10):
        fn()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    for a, b in ev:
        a.record()
        fn()
        b.record()
    torch.cuda.synchronize()
    return float(np.median([a.elapsed_time(b) for a, b in ev])) * 1e3


def main():
    dev = torch.device("cuda:0")
    store = GraphStore(pack_graphs(records(make_dataset(64, seed=1000))), dev)
    h = BatchHandle(store, np.arange(64, dtype=np.int32))
    torch.manual_seed(0)
    model = GINet(30, 1, 3).to(dev).train()
    step = FusedTrainStep(model)
    step.step(h)
    x = torch.zeros(16, device=dev)
    print(f"tiny torch fill kernel      : {timed(lambda: x.fill_(1.0)):7.2f} us")
    print(f"full step (graph + reduce)  : {timed(lambda: step.step(h)):7.2f} us")
    # reduce alone on the partials of the last step
    lib = _lib.load()
    tbl, adam = step._table, step._adam  # noqa: SLF001
    args = (tbl, step.slab.data_ptr(), step.head.data_ptr(), h.B, adam, step.lpg.data_ptr(), 1.0 / h.B, step.loss_out.data_ptr(), _lib.stream_ptr(dev))

    def red():
        _lib.check(lib.dr_reduce_update(*args), "dr_reduce_update")

    print(f"reduce+Adam alone (resident): {timed(red):7.2f} us")


if __name__ == "__main__":
    main()
