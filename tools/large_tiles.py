"""Diagnostic: GINet atom-level step time (config 4 shape) per tile size of
the split path, with and without tile halos in LDS."""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deeprank-gnn-2_amd")]

from bench import make_graphs, records  # noqa: E402
from deeprank2_amd.engine import FusedTrainStep  # noqa: E402
from deeprank2_amd.fused import BatchHandle  # noqa: E402
from deeprank2_amd.neuralnets.gnn.ginet import GINet  # noqa: E402
from deeprank2_amd.store import GraphStore, pack_graphs  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B = 32
    store = GraphStore(pack_graphs(records(make_graphs("atom", B, 1000))), dev)
    torch.manual_seed(0)
    for tile in (128, 96, 64):
        for halos in (True, False):
            step = FusedTrainStep(GINet(30, 1, 3).to(dev).train())
            h = BatchHandle(store, np.arange(B, dtype=np.int32))
            h.large_tile, h.large_halos = tile, halos
            plan = h.large_plan(1)
            g = step.capture(h)
            g.replay()
            torch.cuda.synchronize()
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(30):
                g.replay()
            b.record()
            torch.cuda.synchronize()
            print(f"tile {tile:3d} halos {int(halos)}: {a.elapsed_time(b) / 30 * 1e3:7.1f} us/step  conv LDS {plan.conv_lds} B, tiles {plan.n_tiles}")


if __name__ == "__main__":
    main()
