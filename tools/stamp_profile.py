"""Diagnostic: per-phase cycle shares of ginet_graph_kernel (or
ginet_nocluster_kernel) from the stamps build.

    DR_LIB_NAME=libdeeprank2_amd_stamps.so python tools/stamp_profile.py [B] [ginet|ginet_nocluster]

Stamps (s_memtime, shader clock cycles) are taken by thread 0 right after each
phase barrier; the build that takes them is never used for timing claims —
read the shares, not the absolute length.
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
from deeprank2_amd.neuralnets.gnn import ginet as amd  # noqa: E402
from deeprank2_amd.neuralnets.gnn import ginet_nocluster as amd_nc  # noqa: E402
from deeprank2_amd.store import GraphStore, pack_graphs  # noqa: E402
from deeprank2_amd.utils.synthetic import make_dataset  # noqa: E402

PHASES_NC = ["stage", "gather Z1=AX", "gemm H1", "gather Z2=AH1", "gemm2+bits+colsum", "mean", "head fwd+loss+bwd", "dW2", "dZ2", "spmmT dS1", "dW1"]
PHASES_V = ["stage", "gemm B1", "row fwd 1", "gemm X1", "gemm B2 + hand-off 1", "row fwd 2", "gemm X2", "mean+bits + hand-off 2", "head fwd/loss/bwd", "dWn2, dS2 + hand-off 3", "D2 pass", "row T 2", "dWa2 dWb2 dX1", "DMA X0/S1, dS1 + h-o 4", "dWn1", "D1 pass", "row T 1", "dWa1 dWb1"]
PHASES = ["stage", "front: gather+MFMA+pool0 (per wave)", "front barrier wait", "pool0 key decode", "gemm2+spmm2", "pool1", "mean", "head fwd (fc1,fc2)", "loss grad", "head bwd", "pool1-bwd", "spmm2T", "dW2+dP1", "dW1"]


def main():
    dev = torch.device("cuda:0")
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    which = sys.argv[2] if len(sys.argv) > 2 else "ginet"
    if which == "vanilla":
        return vanilla(dev, B)
    if which in ("foutnet", "sgat"):
        return fout(dev, B, which)
    mod, phases = (amd_nc, PHASES_NC) if which == "ginet_nocluster" else (amd, PHASES)
    large = which == "ginet_large"
    if large:  # tail kernel of the split path on atom-level graphs (stamps 0-3: staging, tile combine; then as ginet_graph_kernel)
        phases = ["stage", "tile combine", "-", *PHASES[3:]]
    fam = {"n_lo": 2700, "n_hi": 3300, "mean_degree": 16.7, "k_lo": 8, "k_hi": 32} if large else {}
    store = GraphStore(pack_graphs(records(make_dataset(B, seed=1000, **fam))), dev)
    h = amd.BatchHandle(store, np.arange(B))
    if large:
        h.large_tile = 64
    torch.manual_seed(0)
    model = mod.GINet(30, 1, 3).to(dev)
    params = model.ordered_params()
    st = torch.zeros(B * 32, dtype=torch.int64, device=dev)
    out = torch.empty(B, 1, device=dev)
    slab = torch.empty(B * amd.slab_stride(30), device=dev)
    head = torch.empty(B * amd.head_stride(1), device=dev)
    lpg = torch.empty(B, device=dev)
    rows, rows_full = [], []
    for it in range(30):
        mod.graph_pass(h, params, 1, 3, dropout=amd.Dropout(0.4, seed=1, offset=it), loss_kind=1, loss_scale=1 / B, out=out, loss_per_graph=lpg, slab=slab, head=head, stamps=st)
        torch.cuda.synchronize()
        if it >= 5:
            rows.append(st.view(B, 32)[:, : len(phases) + 1].cpu().numpy().copy())
            rows_full.append(st.view(B, 32).cpu().numpy().copy())
    a = np.stack(rows)  # [iters, B, 16]
    d = np.diff(a, axis=2).astype(np.float64)  # phase i = stamp[i+1]-stamp[i]
    med = np.median(d.reshape(-1, d.shape[-1]), axis=0)
    tot = med.sum()
    print(f"B={B}  median cycles per graph-kernel workgroup: {tot:.0f}")
    print(which)
    for name, v in zip(phases, med):
        print(f"  {name:18s} {v:8.0f} cyc  {100 * v / tot:5.1f}%")
    if which == "ginet":  # wave 0's first tile inside the front half (stamps 20-22)
        full = np.stack([r for r in rows_full])
        if np.median(full[:, :, 22]) > 0:
            g = np.median(full[:, :, 20] - full[:, :, 1]), np.median(full[:, :, 21] - full[:, :, 20]), np.median(full[:, :, 22] - full[:, :, 21])
            print(f"  wave 0 tile 0: gather {g[0]:.0f}  MFMA {g[1]:.0f}  pool atomics {g[2]:.0f} cyc")


PHASES_F = ["stage", "gather rowmean(X)", "gemm conv1", "pool0", "conv2 (pooled)", "pool1+mean", "head fwd", "loss", "head/pool1/conv2 bwd", "dW1"]


def fout(dev, B, which):
    """fout_graph_kernel (FoutNet, or SGAT with one edge feature) phases on residue graphs."""
    from deeprank2_amd import _lib  # noqa: PLC0415
    from deeprank2_amd.fused import make_pass  # noqa: PLC0415
    from deeprank2_amd.neuralnets.gnn import foutnet, sgat  # noqa: PLC0415

    fe = 1 if which == "sgat" else 3
    store = GraphStore(pack_graphs(records(make_dataset(B, seed=1000), fe)), dev)
    h = amd.BatchHandle(store, np.arange(B))
    torch.manual_seed(0)
    model = (sgat.SGAT if which == "sgat" else foutnet.FoutNet)(30, 1, fe).to(dev)
    spec = model.fused_spec
    st = torch.zeros(B * 32, dtype=torch.int64, device=dev)
    out = torch.empty(B, 1, device=dev)
    slab = torch.empty(B * spec.slab_stride(30), device=dev)
    head = torch.empty(B * spec.head_stride(1), device=dev)
    lpg = torch.empty(B, device=dev)
    params = model.ordered_params()
    rows = []
    for it in range(30):
        p = make_pass(1, _lib.DR_PASS_FORWARD | _lib.DR_PASS_BACKWARD, loss_kind=_lib.DR_LOSS_MSE, loss_scale=1 / B, out=out, loss_per_graph=lpg, slab=slab, head=head, stamps=st)
        from deeprank2_amd.fused import run_pass  # noqa: PLC0415

        run_pass(spec, h, params, p)
        torch.cuda.synchronize()
        if it >= 5:
            rows.append(st.view(B, 32).cpu().numpy().copy())
    full = np.stack(rows)
    d = np.diff(full[:, :, : len(PHASES_F) + 1], axis=2).astype(np.float64)
    med = np.median(d.reshape(-1, d.shape[-1]), axis=0)
    tot = med.sum()
    print(f"B={B}  median cycles per fout_graph_kernel workgroup ({which}): {tot:.0f}")
    for name, v in zip(PHASES_F, med):
        print(f"  {name:22s} {v:8.0f} cyc  {100 * v / tot:5.1f}%")
    if np.median(full[:, :, 22]) > 0:  # wave 0's first tile inside the front half (stamps 20-22)
        g = np.median(full[:, :, 20] - full[:, :, 1]), np.median(full[:, :, 21] - full[:, :, 20]), np.median(full[:, :, 22] - full[:, :, 21])
        print(f"  wave 0 tile 0: gather {g[0]:.0f}  MFMA {g[1]:.0f}  pool atomics {g[2]:.0f} cyc")


def vanilla(dev, B):
    """vanilla_graph_kernel (dr_vanilla_fused_pass) phases on residue graphs,
    per workgroup (DR_SPLIT workgroups per graph, default by batch size); the
    hand-off phases include their waits, reported separately (entry -> done)."""
    from deeprank2_amd import _lib  # noqa: PLC0415
    from deeprank2_amd.fused import make_pass  # noqa: PLC0415
    from deeprank2_amd.neuralnets.gnn import vanilla_gnn as van  # noqa: PLC0415

    store = GraphStore(pack_graphs(records(make_dataset(B, seed=1000))), dev)
    h = amd.BatchHandle(store, np.arange(B))
    if os.environ.get("DR_SPLIT"):
        h.vanilla_split = int(os.environ["DR_SPLIT"])
    k = van.split_k(h, 30, 3)
    torch.manual_seed(0)
    model = van.VanillaNetwork(30, 1, 3).to(dev)
    spec = model.fused_spec
    assert van.fused_fits(h, 30, 3)
    st = torch.zeros(B * k * 32, dtype=torch.int64, device=dev)
    out = torch.empty(B, 1, device=dev)
    slab = torch.empty(B * spec.slab_stride(30), device=dev)
    head = torch.empty(B * spec.head_stride(1), device=dev)
    lpg = torch.empty(B, device=dev)
    w = spec.weights(model.ordered_params())
    rows = []
    for it in range(30):
        p = make_pass(1, _lib.DR_PASS_FORWARD | _lib.DR_PASS_BACKWARD, loss_kind=_lib.DR_LOSS_MSE, loss_scale=1 / B, out=out, loss_per_graph=lpg, slab=slab, head=head, stamps=st)
        spec.run(h, w, p)
        torch.cuda.synchronize()
        if it >= 5:
            rows.append(st.view(B * k, 32).cpu().numpy().copy())
    a = np.stack(rows).astype(np.float64)  # [iters, B*k, 32]
    d = np.diff(a[:, :, : len(PHASES_V) + 1], axis=2)
    med = np.median(d.reshape(-1, d.shape[-1]), axis=0)
    tot = med.sum()
    print(f"B={B} split={k}  median cycles per vanilla_graph_kernel workgroup: {tot:.0f}")
    for name, v in zip(PHASES_V, med):
        print(f"  {name:18s} {v:8.0f} cyc  {100 * v / tot:5.1f}%")
    if k > 1:  # hand-off waits: entry stamp (19..22) -> the next phase stamp
        for name, e, x in (("hand-off 1 (B2)", 19, 5), ("hand-off 2 (col sums)", 20, 8), ("hand-off 3 (dS2)", 21, 10), ("hand-off 4 (dS1)", 22, 14)):
            print(f"  {name:22s} {np.median(a[:, :, x] - a[:, :, e]):8.0f} cyc (wait + gather)")
        if np.median(a[:, :, 24]) > 0:  # d_pass stamps (layer 2): copy, rows of the first segment
            print(f"  D2 copy {np.median(a[:, :, 23] - a[:, :, 10]):8.0f}  rows {np.median(a[:, :, 24] - a[:, :, 23]):8.0f}  rest {np.median(a[:, :, 11] - a[:, :, 24]):8.0f} cyc")
        span = a[:, :, len(PHASES_V)] - a[:, :, 0]
        print(f"  workgroup span min/median/max {span.min():.0f} / {np.median(span):.0f} / {span.max():.0f} cyc")


if __name__ == "__main__":
    main()
