"""Diagnostic: phase stamps of the Vanilla chunk-fused kernels (vc_fwd<1>,
vc_fwd<2>, vc_nb2, vc_eb2n1, vc_eb1) from the stamps build, one training step
of the atom-level (B=32) or mixed (B=64) workload.

    DR_LIB_NAME=libdeeprank2_amd_stamps.so python tools/vchunk_stamps.py [atom|mixed]

Per kernel: the median workgroup lifetime and phase split (thread 0's
s_memtime after each phase barrier).  Only differences of one workgroup's own
stamps are read: s_memtime counters of different CUs / XCDs are not aligned
(spans across workgroups came out as ~1e8 ticks).
The stamps build is never used for timing claims: read the shares.
"""

from __future__ import annotations

import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deeprank-gnn-2_amd")]
os.environ.setdefault("DR_LIB_NAME", "libdeeprank2_amd_stamps.so")

from bench import make_graphs, records  # noqa: E402
from deeprank2_amd.engine import GINetTrainStep  # noqa: E402
from deeprank2_amd.neuralnets.gnn.ginet import BatchHandle  # noqa: E402
from deeprank2_amd.neuralnets.gnn.vanilla_gnn import VanillaNetwork  # noqa: E402
from deeprank2_amd.store import GraphStore, pack_graphs  # noqa: E402
from deeprank2_amd.utils.synthetic import make_dataset  # noqa: E402

KERNELS = [
    ("vc_fwd<1>", ["stage", "[A|B] MFMA", "edge gather", "node MLP"]),
    ("vc_fwd<2>", ["stage", "[A|B] MFMA", "edge gather", "node MLP"]),
    ("vc_nb2", ["stage", "GEMM dX1|DS2 + dWn2"]),
    ("vc_eb2n1", ["stage", "edge bwd", "late rows (DMA)", "dW edge + dX1 GEMM", "DS1 + dWn1"]),
    ("vc_eb1", ["stage", "edge bwd", "X0 (DMA) + dW edge"]),
]


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "atom"
    dev = torch.device("cuda:0")
    if which == "mixed":
        B, graphs = 64, make_graphs("mixed", 64 * 2, seed=1000)
    else:
        B, graphs = 32, make_dataset(64, seed=1000, n_lo=2700, n_hi=3300, mean_degree=16.7, k_lo=8, k_hi=32)
    packed = pack_graphs(records(graphs, 3), require_clusters=False)
    store = GraphStore(packed, dev)
    hs = [BatchHandle(store, np.arange(i * B, (i + 1) * B, dtype=np.int32)) for i in range(2)]
    torch.manual_seed(1234)
    step = GINetTrainStep(VanillaNetwork(30, 1, 3).to(dev).train())
    for i in range(6):
        step.step(hs[i % 2])
    torch.cuda.synchronize()
    n = np.diff(packed.node_off.astype(np.int64))[:B]
    n_tiles = int(((n + 63) // 64).sum())
    st = torch.zeros(5 * n_tiles * 16, dtype=torch.int64, device=dev)
    for p in (step._pass, step._pass_nodrop):  # noqa: SLF001
        p.stamps = st.data_ptr()
    step.step(hs[0])
    torch.cuda.synchronize()
    a = st.view(5, n_tiles, 16).cpu().numpy().astype(np.int64)
    print(f"workload {which}: B={B} chunks={n_tiles} (stamp ticks; shares matter, not absolute length)")
    for k, (name, phases) in enumerate(KERNELS):
        s = a[k]
        if not (s[:, 0] > 0).all():
            print(f"{name}: missing stamps")
            continue
        np_ = len(phases)
        end = s[:, np_]
        life = end - s[:, 0]
        d = np.diff(s[:, : np_ + 1], axis=1)
        med = np.median(d, axis=0)
        parts = ", ".join(f"{ph} {m:.0f} ({100 * m / med.sum():.0f}%)" for ph, m in zip(phases, med))
        print(f"{name}: WG lifetime median {np.median(life):.0f} p90 {np.percentile(life, 90):.0f}; phases: {parts}")
        if name.startswith("vc_eb") and (s[:, 8] > 0).all():  # the edge backward's counts pass (stamp 8) / transposed pass
            print(f"  edge bwd split: counts {np.median(s[:, 8] - s[:, 1]):.0f}, transposed {np.median(s[:, 2] - s[:, 8]):.0f}")


if __name__ == "__main__":
    main()
