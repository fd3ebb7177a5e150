"""Diagnostic: per-phase cycles of the accumulating GINet pass
(ginet_acc_kernel) against the per-graph kernel (ginet_graph_kernel) on the
same batch, from the stamps build.

    DR_LIB_NAME=libdeeprank2_amd_stamps.so python tools/acc_stamps.py [B]

Per graph: the median cycles of each phase (stamps 0..14, s_memtime, thread 0
after each phase barrier) on both kernels; for the accumulating kernel also
the gap between one graph's last stamp and the next graph's first stamp on the
same workgroup (the end-of-graph barrier and the next graph's entry).  The
stamps build is never used for timing claims.
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
from deeprank2_amd.engine import FusedTrainStep  # noqa: E402
from deeprank2_amd.fused import BatchHandle  # noqa: E402
from deeprank2_amd.neuralnets.gnn.ginet import GINet  # noqa: E402
from deeprank2_amd.store import GraphStore, pack_graphs  # noqa: E402

sys.path.insert(0, os.path.join(ROOT, "tools"))
from stamp_profile import PHASES  # noqa: E402


def run(step, h, stamps, iters=12):
    for p in (step._pass, step._pass_nodrop):  # noqa: SLF001
        p.stamps = stamps.data_ptr()
    rows = []
    for i in range(iters):
        stamps.zero_()
        step.step(h)
        torch.cuda.synchronize()
        if i >= 2:
            rows.append(stamps.view(h.B, 32).cpu().numpy().astype(np.float64).copy())
    return np.stack(rows)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    dev = torch.device("cuda:0")
    store = GraphStore(pack_graphs(records(make_graphs("residue", B, seed=1000))), dev)
    h = BatchHandle(store, np.arange(B, dtype=np.int32))
    stamps = torch.zeros(B * 32, dtype=torch.int64, device=dev)
    res = {}
    for mode in ("per-graph", "acc"):
        torch.manual_seed(1234)
        step = FusedTrainStep(GINet(30, 1, 3).to(dev).train(), max_batch=B)
        step.acc = mode == "acc"
        step.acc_prefetch = os.environ.get("DR_ACC_PREFETCH") == "1"
        res[mode] = run(step, h, stamps)
    n = len(PHASES)
    print(f"B={B}  median cycles per graph (s_memtime)")
    print(f"  {'phase':40s} {'per-graph':>10s} {'acc':>10s}")
    meds = {m: np.median(np.diff(a[:, :, : n + 1], axis=2).reshape(-1, n), axis=0) for m, a in res.items()}
    for i, name in enumerate(PHASES):
        print(f"  {name:40s} {meds['per-graph'][i]:10.0f} {meds['acc'][i]:10.0f}")
    print(f"  {'total (stamp 14 - stamp 0)':40s} {meds['per-graph'].sum():10.0f} {meds['acc'].sum():10.0f}")
    # accumulating kernel: the gap between consecutive graphs of one workgroup
    r = min(B, torch.cuda.get_device_properties(dev).multi_processor_count)
    a = res["acc"]
    gaps = []
    for w in range(r):
        g = np.arange(w, B, r)  # workgroup w's graphs (no plan: every r-th position)
        for k in range(1, len(g)):
            gaps.append(a[:, g[k], 0] - a[:, g[k - 1], n])
    gaps = np.concatenate(gaps)
    pf = a[:, :, 16] > 0
    if pf.any():
        d1 = (a[:, :, 17] - a[:, :, 16])[pf]
        d2 = (a[:, :, 18] - a[:, :, 17])[pf]
        d3 = (a[:, :, 4] - a[:, :, 18])[pf]
        print(f"  acc prefetch (wave 0): next descriptor {np.median(d1):.0f} cyc, DMA issue {np.median(d2):.0f} cyc, issue -> tail start {np.median(d3):.0f} cyc")
    print(f"  acc: gap between a workgroup's consecutive graphs: median {np.median(gaps):.0f} cyc, p90 {np.percentile(gaps, 90):.0f}")
    # per-graph kernel: the spread of graph spans (longest / median)
    span = a[:, :, n] - a[:, :, 0]
    span_pg = res["per-graph"][:, :, n] - res["per-graph"][:, :, 0]
    print(f"  graph span median per-graph {np.median(span_pg):.0f} acc {np.median(span):.0f}; p90 {np.percentile(span_pg, 90):.0f} / {np.percentile(span, 90):.0f}")


if __name__ == "__main__":
    main()
