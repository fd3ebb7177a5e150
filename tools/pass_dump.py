"""Diagnostic: one GINet graph pass (forward + backward partials) on seeded
graphs, dumped to .npz, to compare two builds of the library bit for bit
(DR_LIB_NAME selects the build).

    DR_LIB_NAME=libdeeprank2_amd_<v>.so python tools/pass_dump.py <out.npz> [B] [n_lo n_hi]
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deeprank-gnn-2_amd")]

from bench import records  # noqa: E402
from deeprank2_amd.neuralnets.gnn import ginet as amd  # noqa: E402
from deeprank2_amd.store import GraphStore, pack_graphs  # noqa: E402
from deeprank2_amd.utils.synthetic import make_dataset  # noqa: E402


def main():
    path = sys.argv[1]
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 64
    fam = {"n_lo": int(sys.argv[3]), "n_hi": int(sys.argv[4])} if len(sys.argv) > 4 else {}
    dev = torch.device("cuda:0")
    store = GraphStore(pack_graphs(records(make_dataset(B, seed=1000, **fam))), dev)
    h = amd.BatchHandle(store, np.arange(B))
    torch.manual_seed(0)
    model = amd.GINet(30, 1, 3).to(dev)
    params = model.ordered_params()
    out = torch.empty(B, 1, device=dev)
    slab = torch.empty(B * amd.slab_stride(30), device=dev)
    head = torch.empty(B * amd.head_stride(1), device=dev)
    lpg = torch.empty(B, device=dev)
    amd.graph_pass(h, params, 1, 3, dropout=amd.Dropout(0.4, seed=1, offset=0), loss_kind=1, loss_scale=1 / B, out=out, loss_per_graph=lpg, slab=slab, head=head)
    torch.cuda.synchronize()
    n = np.diff(store.packed.node_off)[:B] if hasattr(store, "packed") else None
    np.savez(path, out=out.cpu().numpy(), slab=slab.view(B, -1).cpu().numpy(), head=head.view(B, -1).cpu().numpy(), lpg=lpg.cpu().numpy())
    print("saved", path, "N range", None if n is None else (int(n.min()), int(n.max())))


if __name__ == "__main__":
    main()
