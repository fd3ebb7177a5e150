"""Packed, HBM-resident graph store: the data layout every kernel reads.

A DeepRank2 batch goes through ``GraphDataset.load_one_graph`` (reference
``deeprank2/dataset.py:883-1052``), the PyG ``Collater`` (``trainer.py:541``),
then, inside every forward, ``get_preloaded_cluster`` + ``consecutive_cluster``
+ ``pool_edge`` (``community_pooling.py:23-27,205-212``) and PyG's
``max_pool_x`` (``ginet.py:102-103``).  All of that index work is a pure
function of each graph's static ``edge_index``/``cluster0``/``cluster1``, so it
is done ONCE per graph here, and a mini-batch becomes a list of graph ids:

* CSR by ``edge_index[0]`` (the scatter index of ``ginet.py:58``), stable, so
  each row sums its edges in the same order as ``scatter_add_`` on the CPU;
  its transpose (aliased when the graph is symmetric, which
  ``load_one_graph``'s doubled edges always are);
* depth-0 clusters relabelled densely per graph (what the per-batch offset +
  ``consecutive_cluster`` produce, graph by graph) with member lists in
  ascending node order (torch_scatter ``scatter_max`` keeps the first max);
* the pooled graph of ``pool_edge`` (relabel, drop self loops, coalesce ->
  unique pairs sorted by (row, col)) as a CSR, and its transpose;
* depth-1 clusters relabelled densely with member lists.

Per graph the index arrays use local int32 ids; offsets are int64.
"""

from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np


@dataclass
class GraphRecord:
    """One graph as ``load_one_graph`` returns it (numpy)."""

    x: np.ndarray  # [N, F] float32
    edge_index: np.ndarray  # [2, E] int64 (doubled: both directions)
    edge_attr: np.ndarray | None = None  # [E, Fe] float32
    cluster0: np.ndarray | None = None  # [N] int64
    cluster1: np.ndarray | None = None  # [K0] int64
    y: float | None = None
    pos: np.ndarray | None = None
    name: str = ""


@dataclass
class PackedGraphs:
    n_feat: int
    n_graphs: int
    x: np.ndarray
    node_off: np.ndarray
    edge_off: np.ndarray
    rowptr: np.ndarray
    col: np.ndarray
    eperm: np.ndarray  # CSR slot -> original edge position within the graph
    t_rowptr: np.ndarray
    t_col: np.ndarray
    t_eid: np.ndarray  # transposed CSR slot -> CSR slot of the same edge (local)
    transpose_aliased: bool
    k0_off: np.ndarray
    m0_ptr: np.ndarray
    m0_idx: np.ndarray
    cl0: np.ndarray  # [N_all] dense depth-0 id per node
    p1_off: np.ndarray
    p1_rowptr: np.ndarray
    p1_col: np.ndarray
    p1t_rowptr: np.ndarray
    p1t_col: np.ndarray
    p1t_pid: np.ndarray  # pooled transposed slot -> pooled CSR slot (local)
    k1_off: np.ndarray
    m1_ptr: np.ndarray
    m1_idx: np.ndarray
    cl1: np.ndarray
    y: np.ndarray
    edge_attr: np.ndarray | None  # [E_all, Fe] in CSR order
    p1_ea: np.ndarray | None  # [P1_all, Fe] pooled edge_attr (PyG coalesce: sums of merged edges)
    names: list = field(default_factory=list)
    has_clusters: bool = True  # False: cluster0/1 were missing and filled with one cluster per graph
    # per graph: a non-finite x or edge_attr entry.  GINet's attention
    # (ginet.py:48-54) is identically 1 only for finite logits; such graphs
    # take the layer path, which computes it (layered.ginet_forward)
    nonfinite: np.ndarray | None = None

    # per-graph sizes (host side, for launch geometry)
    def sizes(self):
        n = np.diff(self.node_off)
        e = np.diff(self.edge_off)
        k0 = np.diff(self.k0_off)
        p1 = np.diff(self.p1_off)
        k1 = np.diff(self.k1_off)
        return n, e, k0, p1, k1


def _csr(rows, cols, n):
    perm = np.argsort(rows, kind="stable")
    rowptr = np.zeros(n + 1, dtype=np.int64)
    np.cumsum(np.bincount(rows, minlength=n), out=rowptr[1:])
    return rowptr.astype(np.int32), cols[perm].astype(np.int32), perm.astype(np.int32)


def _same_multiset(r1, c1, r2, c2, n):
    if r1.size != r2.size:
        return False
    a = np.sort(r1.astype(np.int64) * n + c1)
    b = np.sort(r2.astype(np.int64) * n + c2)
    return bool(np.array_equal(a, b))


def _dense(ids, what):
    ids = np.asarray(ids, dtype=np.int64)
    if ids.size and ids.min() < 0:
        msg = f"{what} ids must be non-negative (get_preloaded_cluster offsets assume it)"
        raise ValueError(msg)
    uniq, inv = np.unique(ids, return_inverse=True)
    return inv.astype(np.int64), int(uniq.size)


def pack_graphs(records: list[GraphRecord], require_clusters: bool = True, threads: int = 0) -> PackedGraphs:
    """Pack per-graph records into the store layout with the native host
    packer (``dr_pack_sizes`` / ``dr_pack_fill``, threads over graphs)."""
    import ctypes  # noqa: PLC0415

    from deeprank2_amd import _lib  # noqa: PLC0415

    if not records:
        msg = "empty graph list"
        raise ValueError(msg)
    G = len(records)
    F = int(np.asarray(records[0].x).shape[1])
    xs, eis, c0s, c1s, ys, eas = [], [], [], [], [], []
    node_off = np.zeros(G + 1, np.int64)
    edge_off = np.zeros(G + 1, np.int64)
    c1_off = np.zeros(G + 1, np.int64)
    has_ea = records[0].edge_attr is not None
    has_clusters = all(r.cluster0 is not None and r.cluster1 is not None for r in records)
    if require_clusters and not has_clusters:
        g = next(i for i, r in enumerate(records) if r.cluster0 is None or r.cluster1 is None)
        msg = f"graph {g} ({records[g].name}) has no cluster0/cluster1 (set clustering_method when building the dataset)"
        raise ValueError(msg)
    for gi, r in enumerate(records):
        x = np.asarray(r.x, dtype=np.float32)
        if x.ndim != 2 or x.shape[1] != F:
            msg = f"graph {gi}: x must be [N, {F}]"
            raise ValueError(msg)
        n = x.shape[0]
        ei = np.asarray(r.edge_index, dtype=np.int64).reshape(2, -1)
        xs.append(x)
        eis.append(ei)
        node_off[gi + 1] = node_off[gi] + n
        edge_off[gi + 1] = edge_off[gi] + ei.shape[1]
        if has_clusters:
            c0 = np.asarray(r.cluster0, dtype=np.int64).reshape(-1)
            if len(c0) != n:
                msg = f"graph {gi}: cluster0 has {len(c0)} entries for {n} nodes"
                raise ValueError(msg)
            c1 = np.asarray(r.cluster1, dtype=np.int64).reshape(-1)
            c0s.append(c0)
            c1s.append(c1)
            c1_off[gi + 1] = c1_off[gi] + len(c1)
        ys.append(np.nan if r.y is None else float(np.asarray(r.y).reshape(-1)[0]))
        if has_ea:
            eas.append(np.asarray(r.edge_attr, dtype=np.float32).reshape(ei.shape[1], -1))
    x = np.concatenate(xs) if G else np.zeros((0, F), np.float32)
    ei_all = np.ascontiguousarray(np.concatenate(eis, axis=1)) if G else np.zeros((2, 0), np.int64)
    ea_all = np.ascontiguousarray(np.concatenate(eas)) if has_ea else None
    fe = 0 if ea_all is None else ea_all.shape[1]
    c0_all = np.ascontiguousarray(np.concatenate(c0s)) if has_clusters else None
    c1_all = np.ascontiguousarray(np.concatenate(c1s)) if has_clusters else None

    lib = _lib.load()
    P = lambda a: None if a is None else a.ctypes.data  # noqa: E731
    inp = _lib.PackInputC()
    inp.n_graphs, inp.n_feat, inp.n_edge_feat, inp.require_clusters = G, F, fe, int(require_clusters)
    inp.node_off, inp.edge_off, inp.c1_off = P(node_off), P(edge_off), P(c1_off)
    inp.edge_index, inp.edge_attr, inp.cluster0, inp.cluster1 = P(ei_all), P(ea_all), P(c0_all), P(c1_all)
    k0c, p1c, k1c = np.zeros(G, np.int64), np.zeros(G, np.int64), np.zeros(G, np.int64)
    sym = ctypes.c_int32(0)
    err = ctypes.create_string_buffer(256)
    rc = lib.dr_pack_sizes(inp, P(k0c), P(p1c), P(k1c), threads, err, 256)
    if rc != 0:
        raise ValueError(err.value.decode() or "invalid graphs")
    k0_off = np.concatenate([[0], np.cumsum(k0c)]).astype(np.int64)
    p1_off = np.concatenate([[0], np.cumsum(p1c)]).astype(np.int64)
    k1_off = np.concatenate([[0], np.cumsum(k1c)]).astype(np.int64)
    N, E, K0, P1, K1 = int(node_off[-1]), int(edge_off[-1]), int(k0_off[-1]), int(p1_off[-1]), int(k1_off[-1])
    i32 = lambda m: np.empty(max(m, 0), np.int32)  # noqa: E731
    out = {
        "rowptr": i32(N + G), "col": i32(E), "eperm": i32(E), "t_rowptr": i32(N + G), "t_col": i32(E), "t_eid": i32(E),
        "m0_ptr": i32(K0 + G), "m0_idx": i32(N), "cl0": i32(N), "p1_rowptr": i32(K0 + G), "p1_col": i32(P1),
        "p1t_rowptr": i32(K0 + G), "p1t_col": i32(P1), "p1t_pid": i32(P1), "m1_ptr": i32(K1 + G), "m1_idx": i32(K0), "cl1": i32(K0),
    }  # fmt: skip
    ea_csr = np.empty((E, fe), np.float32) if fe else None
    p1_ea = np.empty((P1, fe), np.float32) if fe else None
    o = _lib.PackOutputC()
    o.k0_off, o.p1_off, o.k1_off = P(k0_off), P(p1_off), P(k1_off)
    for name, arr in out.items():
        setattr(o, name, P(arr))
    o.edge_attr = P(ea_csr)
    o.p1_ea = P(p1_ea)
    _lib.check(lib.dr_pack_fill(inp, o, ctypes.addressof(sym), threads), "dr_pack_fill")
    return PackedGraphs(
        nonfinite=nonfinite_graphs(x, node_off, ea_all, edge_off),
        n_feat=F,
        n_graphs=G,
        x=x,
        node_off=node_off,
        edge_off=edge_off,
        transpose_aliased=bool(sym.value),
        k0_off=k0_off,
        p1_off=p1_off,
        k1_off=k1_off,
        y=np.asarray(ys, dtype=np.float32),
        edge_attr=ea_csr if has_ea else None,
        p1_ea=p1_ea if has_ea else None,
        names=[r.name for r in records],
        has_clusters=has_clusters,
        **out,
    )


def nonfinite_graphs(x, node_off, edge_attr=None, edge_off=None) -> np.ndarray:
    """bool [G]: graph g holds a non-finite node feature or edge attribute."""
    G = node_off.size - 1
    bad = np.zeros(G, bool)
    for a, off in ((x, node_off), (edge_attr, edge_off)):
        if a is None or a.size == 0 or np.isfinite(a).all():  # (one flat pass: the common, finite case)
            continue
        rows = np.flatnonzero(~np.isfinite(a.reshape(a.shape[0], -1)).all(axis=1))
        if rows.size:
            bad[np.searchsorted(off, rows, side="right") - 1] = True
    return bad


def records_from_batch(batch) -> list[GraphRecord]:
    """Split a collated PyG-style batch (x, edge_index, batch/ptr, cluster0,
    cluster1, edge_attr, y) back into per-graph records (host side)."""
    import torch  # noqa: PLC0415

    def np_(t):
        return None if t is None else (t.detach().cpu().numpy() if isinstance(t, torch.Tensor) else np.asarray(t))

    x = np_(batch.x)
    ei = np_(batch.edge_index)
    ea = np_(getattr(batch, "edge_attr", None))
    bvec = np_(getattr(batch, "batch", None))
    if bvec is None:
        bvec = np.zeros(x.shape[0], dtype=np.int64)
    n_graphs = int(bvec.max()) + 1 if bvec.size else 0
    counts = np.bincount(bvec, minlength=n_graphs)
    if not np.all(np.diff(bvec) >= 0):
        msg = "batch vector must be sorted (PyG collate order)"
        raise ValueError(msg)
    ptr = np.concatenate([[0], np.cumsum(counts)])
    c0 = np_(getattr(batch, "cluster0", None))
    c1 = np_(getattr(batch, "cluster1", None))
    y = np_(getattr(batch, "y", None))
    names = getattr(batch, "entry_names", None)
    eg = bvec[ei[0]] if ei.size else np.zeros(0, np.int64)
    if ei.size and not np.array_equal(eg, bvec[ei[1]]):
        msg = "edges must not cross graphs"
        raise ValueError(msg)
    eorder = np.argsort(eg, kind="stable")
    ecount = np.bincount(eg, minlength=n_graphs)
    eptr = np.concatenate([[0], np.cumsum(ecount)])
    # cluster1 belongs to depth-0 clusters; split it by each graph's cluster count
    k0s = [len(np.unique(c0[ptr[g]:ptr[g + 1]])) for g in range(n_graphs)] if c0 is not None else None
    kptr = np.concatenate([[0], np.cumsum(k0s)]) if k0s is not None else None
    recs = []
    for g in range(n_graphs):
        sl = slice(ptr[g], ptr[g + 1])
        es = eorder[eptr[g]:eptr[g + 1]]
        recs.append(
            GraphRecord(
                x=x[sl],
                edge_index=ei[:, es] - ptr[g],
                edge_attr=None if ea is None else ea[es],
                cluster0=None if c0 is None else c0[sl],
                cluster1=None if (c1 is None or kptr is None) else c1[kptr[g]:kptr[g + 1]],
                y=None if y is None or y.size <= g else float(y.reshape(-1)[g]),
                name=names[g] if isinstance(names, list) and g < len(names) else f"g{g}",
            ),
        )
    return recs


DESC_DTYPE = np.dtype([("node0", "<i8"), ("col0", "<i8"), ("k0", "<i8"), ("p1", "<i8"), ("k1", "<i8"), ("n_nodes", "<i4"), ("n_edges", "<i4"), ("n_k0", "<i4"), ("n_p1", "<i4"), ("n_k1", "<i4"), ("gid", "<i4")])
assert DESC_DTYPE.itemsize == 64  # dr_graph_desc


class GraphStore:
    """Device copy of a :class:`PackedGraphs` (all arrays live in HBM)."""

    def __init__(self, packed: PackedGraphs, device, dtype: str = "f32"):
        import torch  # noqa: PLC0415

        if dtype not in ("f32", "bf16"):
            msg = f"dtype must be 'f32' or 'bf16' (got {dtype!r})"
            raise ValueError(msg)
        self.dtype = dtype

        self.packed = packed
        self.device = torch.device(device)
        t = lambda a: torch.from_numpy(np.ascontiguousarray(a)).to(self.device)  # noqa: E731
        p = packed
        # Device layout: x rows padded to a multiple of 4 floats (16-byte rows,
        # zero pad) and each graph's col / t_col block 16-byte aligned, so the
        # kernels stage them with 16-byte global->LDS DMA.
        self.x_stride = (p.n_feat + 3) & ~3
        xp = np.zeros((p.x.shape[0], self.x_stride), dtype=np.float32)
        xp[:, : p.n_feat] = p.x
        self.x = t(xp)
        # bf16 compute (dr_pass.compute_dtype): a bf16 copy of x, rows padded to
        # 8 values (16 bytes), rounded to nearest even by torch
        self.x_bf16_stride = (p.n_feat + 7) & ~7
        self.x_bf16 = None
        if dtype == "bf16":
            xb = torch.zeros((p.x.shape[0], self.x_bf16_stride), dtype=torch.bfloat16)
            xb[:, : p.n_feat] = torch.from_numpy(np.ascontiguousarray(p.x, dtype=np.float32)).to(torch.bfloat16)
            self.x_bf16 = xb.to(self.device)
        self.node_off = t(p.node_off)
        self.edge_off = t(p.edge_off)
        if np.diff(p.node_off).max() > 65535:
            msg = "graphs with more than 65535 nodes are not supported (16-bit local column ids)"
            raise ValueError(msg)
        ecount = np.diff(p.edge_off)
        col_off = np.zeros(p.n_graphs + 1, dtype=np.int64)
        np.cumsum((ecount + 7) & ~7, out=col_off[1:])  # 16-byte aligned uint16 blocks
        self.col_off_host = col_off
        self.col_off = t(col_off)
        # gather index: graph g's CSR slot e lives at col_off[g] + e
        slot = np.arange(int(p.edge_off[-1]), dtype=np.int64) - np.repeat(p.edge_off[:-1], ecount) + np.repeat(col_off[:-1], ecount)

        def spread(a):
            out = np.zeros(max(int(col_off[-1]), 8), dtype=np.uint16)
            out[slot] = a
            return out

        self.rowptr = t(p.rowptr)
        self.col = t(spread(p.col))
        # level-0 transpose in true edge order (by edge_index[1], stable), with
        # t_eid mapping each transposed slot to the CSR slot of the same edge
        self.t_rowptr, self.t_col = t(p.t_rowptr), t(spread(p.t_col))
        teid = np.zeros(max(int(col_off[-1]), 8), dtype=np.int32)
        teid[slot] = p.t_eid
        self.t_eid = t(teid)
        self.n_edge_feat = 0 if p.edge_attr is None else int(p.edge_attr.shape[1])
        ea = np.zeros((max(int(col_off[-1]), 8), max(self.n_edge_feat, 1)), dtype=np.float32)
        if self.n_edge_feat:
            ea[slot] = p.edge_attr
        self.ea = t(ea)
        self.k0_off = t(p.k0_off)
        self.m0_ptr = t(p.m0_ptr)
        self.m0_idx = t(p.m0_idx)
        self.cl0 = t(np.ascontiguousarray(p.cl0, dtype=np.int32))
        self.p1_off = t(p.p1_off)
        self.p1_rowptr = t(p.p1_rowptr)
        self.p1_col = t(p.p1_col if p.p1_col.size else np.zeros(1, np.int32))
        if p.transpose_aliased:
            self.p1t_rowptr, self.p1t_col = self.p1_rowptr, self.p1_col
        else:
            self.p1t_rowptr = t(p.p1t_rowptr)
            self.p1t_col = t(p.p1t_col if p.p1t_col.size else np.zeros(1, np.int32))
        self.p1t_pid = t(p.p1t_pid if p.p1t_pid.size else np.zeros(1, np.int32))
        pea = np.zeros((max(int(p.p1_off[-1]), 1), max(self.n_edge_feat, 1)), dtype=np.float32)
        if self.n_edge_feat and p.p1_ea is not None:
            pea[: p.p1_ea.shape[0]] = p.p1_ea
        self.p1_ea = t(pea)
        self.k1_off = t(p.k1_off)
        self.m1_ptr = t(p.m1_ptr)
        self.m1_idx = t(p.m1_idx)
        self.y = t(p.y)
        self.edge_attr = None if p.edge_attr is None else t(p.edge_attr)
        self._sizes = p.sizes()
        self._c = None

    @property
    def n_graphs(self):
        return self.packed.n_graphs

    @property
    def n_feat(self):
        return self.packed.n_feat

    def set_targets(self, y):
        """Replace the per-graph targets (e.g. class indices for CE)."""
        import torch  # noqa: PLC0415

        self.y = torch.as_tensor(np.asarray(y, np.float32)).to(self.device)
        self._c = None

    def cstruct(self):
        from deeprank2_amd import _lib  # noqa: PLC0415

        if self._c is None:
            s = _lib.GraphStoreC()
            s.n_graphs = self.n_graphs
            s.n_feat = self.n_feat
            s.x_stride = self.x_stride
            s.transpose_aliased = int(self.packed.transpose_aliased)
            for name in ("x", "node_off", "edge_off", "col_off", "rowptr", "col", "t_rowptr", "t_col", "k0_off", "m0_ptr", "m0_idx", "p1_off", "p1_rowptr", "p1_col", "p1t_rowptr", "p1t_col", "k1_off", "m1_ptr", "m1_idx", "y", "ea", "t_eid", "p1_ea", "p1t_pid", "cl0"):
                setattr(s, name, getattr(self, name).data_ptr())
            s.n_edge_feat = self.n_edge_feat
            if self.x_bf16 is not None:
                s.x_bf16 = self.x_bf16.data_ptr()
                s.x_bf16_stride = self.x_bf16_stride
            self._c = s
        return self._c

    def descriptors(self, gids_host):
        """dr_graph_desc records (64 bytes each) for these graph ids, as a device uint8 tensor."""
        import torch  # noqa: PLC0415

        p = self.packed
        g = np.asarray(gids_host, dtype=np.int64)
        d = np.zeros(g.size, dtype=DESC_DTYPE)
        d["node0"] = p.node_off[g]
        d["col0"] = self.col_off_host[g]
        d["k0"] = p.k0_off[g]
        d["p1"] = p.p1_off[g]
        d["k1"] = p.k1_off[g]
        n, e, k0, p1, k1 = self._sizes
        d["n_nodes"], d["n_edges"], d["n_k0"], d["n_p1"], d["n_k1"] = n[g], e[g], k0[g], p1[g], k1[g]
        d["gid"] = g
        return torch.from_numpy(d.view(np.uint8)).to(self.device)

    def max_sizes(self, gids_host):
        n, e, k0, p1, k1 = self._sizes
        g = np.asarray(gids_host, dtype=np.int64)
        return int(n[g].max()), int(e[g].max()), int(k0[g].max()), int(p1[g].max()), int(k1[g].max())

    def edges_in(self, gids_host):
        n, e, *_ = self._sizes
        return int(e[np.asarray(gids_host, dtype=np.int64)].sum())
