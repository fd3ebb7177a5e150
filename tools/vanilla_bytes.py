"""Byte attribution of the VanillaNetwork chunk pipeline:
per kernel and per array, the bytes each launch must move at least — every
array element it reads or writes once, halo rows once per tile that stages
them — for the workloads tools/pmc_run.py profiles (vanilla_atom: B = 32
atom-level graphs; vanilla_mixed: B = 64 of the configs[4] mix), from the
tile plan the pipeline runs (the same cut as fused.vanilla_tile_plan: 64-row
tiles, halo = the union of a tile's out- and in-neighbours).  CPU only.

    python tools/vanilla_bytes.py [vanilla_atom|vanilla_mixed] [pmc_per_kernel table]

With a committed per-kernel PMC table the measured WRITE bytes (exact for
16-byte stores, MI355X_MICROARCH.md §HBM) and FETCH bytes (both as counted
and with the x2 gfx950 correction for wide coalesced reads) stand beside the
attribution.
"""

from __future__ import annotations

import os
import re
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "deeprank-gnn-2_amd")]

from bench import make_graphs, records  # noqa: E402
from deeprank2_amd.store import pack_graphs  # noqa: E402
from deeprank2_amd.utils.synthetic import make_dataset  # noqa: E402

WR = 64  # rows per chunk (DR_VANILLA_CHUNK)


def tiles(packed, gids):
    """(nr, H, ne, nq) per 64-row tile of the batch, graph by graph."""
    out = []
    for gid in gids:
        n0, e0, e1 = int(packed.node_off[gid]), int(packed.edge_off[gid]), int(packed.edge_off[gid + 1])
        ng = int(packed.node_off[gid + 1]) - n0
        rp = packed.rowptr[n0 + gid : n0 + gid + ng + 1].astype(np.int64)
        trp = packed.t_rowptr[n0 + gid : n0 + gid + ng + 1].astype(np.int64)
        col, tcol = packed.col[e0:e1], packed.t_col[e0:e1]
        for r0 in range(0, ng, WR):
            r1 = min(ng, r0 + WR)
            cs, ts = col[rp[r0] : rp[r1]], tcol[trp[r0] : trp[r1]]
            out.append((r1 - r0, np.union1d(cs, ts).size, cs.size, ts.size))
    return np.array(out, dtype=np.int64)


def attribution(t, F=30, Fe=3, B=32):
    """{kernel: [(array, bytes read, bytes written)]} for one step."""
    XS = (F + 3) & ~3
    row = 4 * XS  # a feature row (128 B at F = 30)
    row32 = 128  # a 32-channel row (S, dS)
    nr, H, ne, nq = (t[:, k].sum() for k in range(4))
    n_t = len(t)
    KE, KN = 2 * F + Fe, F + 32
    edge_part = 4 * (32 * KE + 32)  # dWe + dbe of one layer, per chunk
    node_part = 4 * (F * KN + F)  # dWn + dbn
    part_row = 4 * (((32 * KE + 32 + F * KN + F) + 3) & ~3)
    w_fwd = 4 * (32 * KE + 32 + F * KN + F)  # one layer's weights, staged by every tile
    A = {}
    for layer in (1, 2):
        src = "x (store)" if layer == 1 else "X1"
        A[f"vc_fwd<{layer}>"] = [
            (f"{src}: own rows", nr * row, 0),
            (f"{src}: halo rows (once per tile)", H * row, 0),
            ("halo ids", 4 * H, 0),
            ("rowptr", 4 * (nr + n_t), 0),
            ("lcol (uint16)", 2 * ne, 0),
            ("edge_attr", 4 * Fe * ne, 0),
            ("weights (per tile)", n_t * w_fwd, 0),
            (f"S{layer}", 0, nr * row32),
            (f"X{layer}", 0, nr * 4 * F),
            (f"ReLU words L{layer}", 0, 4 * ne),
        ] + ([("column sums (part_mean)", 0, n_t * 128)] if layer == 2 else [])
    A["vc_nb2"] = [
        ("X2, X1 own rows", 2 * nr * row, 0),
        ("S2 own rows", nr * row32, 0),
        ("Wn2 (per tile)", n_t * 4 * F * KN, 0),
        ("dX1", 0, nr * 4 * F),
        ("DS2", 0, nr * row32),
        ("dWn2/dbn2 chunk partials", 0, n_t * node_part),
    ]
    bwd_common = lambda ds: [  # noqa: E731
        (f"{ds}: halo rows (once per tile)", H * row32, 0),
        (f"{ds}: own rows", nr * row32, 0),
        ("halo ids", 4 * H, 0),
        ("rowptr + t_rowptr", 8 * (nr + n_t), 0),
        ("ReLU words (CSR)", 4 * ne, 0),
        ("ReLU words (transposed, via t_eid)", 4 * nq, 0),
        ("edge_attr", 4 * Fe * ne, 0),
        ("ltcol (uint16) + t_eid", 6 * nq, 0),
    ]
    A["vc_eb2n1"] = bwd_common("DS2") + [
        ("X1, dX1, X0 own rows", 3 * nr * row, 0),
        ("S1 own rows", nr * row32, 0),
        ("We2, Wn1 (per tile)", n_t * 4 * (32 * KE + F * 32), 0),
        ("layer-2 edge partials", 0, n_t * edge_part),
        ("DS1", 0, nr * row32),
        ("layer-1 node partials", 0, n_t * node_part),
    ]
    A["vc_eb1"] = bwd_common("DS1") + [
        ("X0 own rows", nr * row, 0),
        ("layer-1 edge partials", 0, n_t * edge_part),
    ]
    A["vc_combine"] = [("chunk partial rows, both layers", 2 * n_t * part_row, 0), ("per-graph slab", 0, B * 2 * 4 * (32 * KE + 32 + F * KN + F))]
    return A, dict(nr=int(nr), H=int(H), ne=int(ne), nq=int(nq), tiles=n_t)


def measured(path):
    """{kernel: (FETCH bytes as counted, WRITE bytes)} from a pmc_per_kernel table."""
    out = {}
    for line in open(path):
        m = re.match(r"(vc_\w+(?:<[^>]*>)?)\s+\d+\s+[\d.]+\s+([\d.]+)\s+([\d.]+)", line)
        if m:
            k = re.sub(r"<3>$", "", m.group(1).replace(" ", ""))
            k = {"vc_fwd<3,1>": "vc_fwd<1>", "vc_fwd<3,2>": "vc_fwd<2>"}.get(k, k)
            out[k] = (float(m.group(2)) * 1024, float(m.group(3)) * 1024)
    return out


def main():
    which = sys.argv[1] if len(sys.argv) > 1 else "vanilla_atom"
    pmc = sys.argv[2] if len(sys.argv) > 2 else None
    atom = which.endswith("_atom")
    B, nb = (32, 4) if atom else (64, 4)
    fam = {"n_lo": 2700, "n_hi": 3300, "mean_degree": 16.7, "k_lo": 8, "k_hi": 32}
    graphs = make_dataset(B * nb, seed=1000, **fam) if atom else make_graphs("mixed", B * nb, seed=1000)
    packed = pack_graphs(records(graphs, 3), require_clusters=False)
    order = np.random.default_rng(0).permutation(packed.n_graphs).astype(np.int32)
    per_batch = [attribution(tiles(packed, order[i * B : (i + 1) * B]), B=B) for i in range(nb)]
    kernels = list(per_batch[0][0].keys())
    meas = measured(pmc) if pmc else {}
    shape = {k: float(np.mean([p[1][k] for p in per_batch])) for k in per_batch[0][1]}
    print(f"{which}: B={B}, mean over the {nb} batches tools/pmc_run.py cycles; per step: " + ", ".join(f"{k} {v:,.0f}" for k, v in shape.items()))
    print(f"{'kernel / array':58s} {'read MB':>9s} {'write MB':>9s}")
    tot_r = tot_w = 0.0
    for k in kernels:
        rows = per_batch[0][0][k]
        rd = [np.mean([p[0][k][i][1] for p in per_batch]) for i in range(len(rows))]
        wr = [np.mean([p[0][k][i][2] for p in per_batch]) for i in range(len(rows))]
        kr, kw = sum(rd), sum(wr)
        tot_r += kr
        tot_w += kw
        m = meas.get(k)
        extra = "" if m is None else f"   measured: FETCH {m[0] / 1e6:.1f} (x2: {2 * m[0] / 1e6:.1f}), WRITE {m[1] / 1e6:.1f}"
        print(f"{k:58s} {kr / 1e6:9.2f} {kw / 1e6:9.2f}{extra}")
        for (name, _, _), r, w in zip(rows, rd, wr):
            print(f"    {name:54s} {r / 1e6:9.2f} {w / 1e6:9.2f}")
    print(f"{'total (graph-pass chunk kernels)':58s} {tot_r / 1e6:9.2f} {tot_w / 1e6:9.2f}   = {(tot_r + tot_w) / 1e6:.1f} MB")
    if meas:
        f = sum(v[0] for v in meas.values())
        w = sum(v[1] for v in meas.values())
        print(f"measured (same kernels): FETCH {f / 1e6:.1f} MB as counted ({2 * f / 1e6:.1f} with x2), WRITE {w / 1e6:.1f} MB")


if __name__ == "__main__":
    main()
