"""Diagnostic: phase stamps of the one-launch GINet step (dr_ginet_train_step)
from the stamps build: per workgroup, the tail's end (stamp 14), the
arrival (16), the reducers' poll + acquire (17) and each reduce pass (18+).

    DR_LIB_NAME=libdeeprank2_amd_stamps.so python tools/step_stamps.py [B]
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deeprank-gnn-2_amd")]
os.environ.setdefault("DR_LIB_NAME", "libdeeprank2_amd_stamps.so")

from bench import records  # noqa: E402
from deeprank2_amd.engine import FusedTrainStep  # noqa: E402
from deeprank2_amd.fused import BatchHandle  # noqa: E402
from deeprank2_amd.neuralnets.gnn.ginet import GINet  # noqa: E402
from deeprank2_amd.store import GraphStore, pack_graphs  # noqa: E402
from deeprank2_amd.utils.synthetic import make_dataset  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    dev = torch.device("cuda:0")
    store = GraphStore(pack_graphs(records(make_dataset(B, seed=1000))), dev)
    h = BatchHandle(store, np.arange(B, dtype=np.int32))
    torch.manual_seed(0)
    model = GINet(30, 1, 3).to(dev).train()
    step = FusedTrainStep(model)
    step.fuse_update = True
    NRMAX = 128  # reducer workgroups follow the B graph workgroups (stamps rows B..)
    st = torch.zeros((B + NRMAX) * 32, dtype=torch.int64, device=dev)
    step._pass.stamps = st.data_ptr()  # noqa: SLF001
    rows = []
    for _ in range(30):
        st.zero_()
        step.step(h)
        torch.cuda.synchronize()
        rows.append(st.view(B + NRMAX, 32).cpu().numpy().copy())
    r = np.stack(rows[5:])  # [it, B+NRMAX, 32]
    g, red = r[:, :B], r[:, B:]
    nr = int((red[0, :, 0] > 0).sum())
    print(f"B={B}, {nr} reducer workgroups; cycles (median over workgroups and iterations)")
    rel = g - g[:, :, 0:1]
    for c, name in [(1, "staged"), (3, "front done"), (14, "tail done")]:
        print(f"  graph WG {name:22s} {np.median(rel[:, :, c]):9.0f}")
    live = red[:, :nr]
    wait = live[:, :, 1] - live[:, :, 0]
    work = live[:, :, 2] - live[:, :, 1]
    print(f"  reducer start -> past poll     {np.median(wait):9.0f}  (max {wait.max():.0f})")
    print(f"  reducer reduce + Adam          {np.median(work):9.0f}  (max {work.max():.0f})")


if __name__ == "__main__":
    main()
