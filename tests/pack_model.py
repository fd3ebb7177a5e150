"""Pure-numpy model of the host packer (``dr_pack_sizes`` / ``dr_pack_fill``,
``deeprank-gnn-2_amd/csrc/pack.cpp``): TEST INFRASTRUCTURE, the checker the
native packer is compared against (tests/test_store.py)."""

from __future__ import annotations

import numpy as np

from deeprank2_amd.store import PackedGraphs, _csr, _dense, _same_multiset


def pack_graphs_numpy(records, require_clusters: bool = True) -> PackedGraphs:  # noqa: PLR0915, C901
    if not records:
        msg = "empty graph list"
        raise ValueError(msg)
    F = int(records[0].x.shape[1])
    xs, rps, cols, eperms, trps, tcols, teids = [], [], [], [], [], [], []
    m0ps, m0is, cl0s, p1rps, p1cs, p1trps, p1tcs, m1ps, m1is, cl1s, ys, eas = ([] for _ in range(12))
    p1tps, p1eas = [], []
    node_off = [0]
    edge_off = [0]
    k0_off = [0]
    p1_off = [0]
    k1_off = [0]
    aliased = True
    has_clusters = True
    has_ea = records[0].edge_attr is not None
    for gi, r in enumerate(records):
        x = np.ascontiguousarray(r.x, dtype=np.float32)
        if x.ndim != 2 or x.shape[1] != F:
            msg = f"graph {gi}: x must be [N, {F}]"
            raise ValueError(msg)
        n = x.shape[0]
        if n == 0:
            msg = f"graph {gi} has no nodes (torch.max over an empty cluster would fail in the reference)"
            raise ValueError(msg)
        ei = np.asarray(r.edge_index, dtype=np.int64).reshape(2, -1)
        e = ei.shape[1]
        if e and (ei.min() < 0 or ei.max() >= n):
            msg = f"graph {gi}: edge_index out of range [0, {n})"
            raise ValueError(msg)
        row, col = ei[0], ei[1]
        rp, cs, perm = _csr(row, col, n)
        trp, tcs, tperm = _csr(col, row, n)
        inv = np.empty(e, dtype=np.int32)
        inv[perm] = np.arange(e, dtype=np.int32)
        teids.append(inv[tperm])
        sym = _same_multiset(row, col, col, row, n)
        aliased &= sym
        xs.append(x)
        rps.append(rp)
        cols.append(cs)
        eperms.append(perm)
        trps.append(trp)
        tcols.append(tcs)
        if has_ea:
            ea = np.asarray(r.edge_attr, dtype=np.float32).reshape(e, -1)
            eas.append(ea[perm])

        if r.cluster0 is None or r.cluster1 is None:
            if require_clusters:
                msg = f"graph {gi} ({r.name}) has no cluster0/cluster1 (set clustering_method when building the dataset)"
                raise ValueError(msg)
            c0 = np.zeros(n, dtype=np.int64)
            c1 = np.zeros(1, dtype=np.int64)
            has_clusters = False
        else:
            c0, c1 = r.cluster0, r.cluster1
        if len(c0) != n:
            msg = f"graph {gi}: cluster0 has {len(c0)} entries for {n} nodes"
            raise ValueError(msg)
        d0, k0 = _dense(c0, "cluster0")
        m0i = np.argsort(d0, kind="stable").astype(np.int32)
        m0p = np.zeros(k0 + 1, dtype=np.int32)
        np.cumsum(np.bincount(d0, minlength=k0), out=m0p[1:])
        # pool_edge: relabel, remove self loops, coalesce (unique, sorted by (row, col))
        pr, pc = d0[row], d0[col]
        keep = pr != pc
        key = np.unique(pr[keep] * k0 + pc[keep])
        prow, pcol = key // k0, key % k0
        p1rp = np.zeros(k0 + 1, dtype=np.int32)
        np.cumsum(np.bincount(prow, minlength=k0), out=p1rp[1:])
        tkey = np.unique(pcol * k0 + prow)
        p1tps.append(np.searchsorted(key, (tkey % k0) * k0 + tkey // k0).astype(np.int32))
        if has_ea:  # PyG coalesce: attributes of merged edges summed in edge order
            ea_in = np.asarray(r.edge_attr, dtype=np.float32).reshape(e, -1)
            pe = np.zeros((key.size, ea_in.shape[1]), np.float32)
            np.add.at(pe, np.searchsorted(key, pr[keep] * k0 + pc[keep]), ea_in[keep])
            p1eas.append(pe)
        p1trp = np.zeros(k0 + 1, dtype=np.int32)
        np.cumsum(np.bincount(tkey // k0, minlength=k0), out=p1trp[1:])

        c1 = np.asarray(c1, dtype=np.int64).reshape(-1)
        if len(c1) != k0:
            msg = f"graph {gi}: cluster1 has {len(c1)} entries but cluster0 defines {k0} clusters"
            raise ValueError(msg)
        d1, k1 = _dense(c1, "cluster1")
        m1i = np.argsort(d1, kind="stable").astype(np.int32)
        m1p = np.zeros(k1 + 1, dtype=np.int32)
        np.cumsum(np.bincount(d1, minlength=k1), out=m1p[1:])

        m0ps.append(m0p)
        m0is.append(m0i)
        cl0s.append(d0.astype(np.int32))
        p1rps.append(p1rp)
        p1cs.append(pcol.astype(np.int32))
        p1trps.append(p1trp)
        p1tcs.append((tkey % k0).astype(np.int32))
        m1ps.append(m1p)
        m1is.append(m1i)
        cl1s.append(d1.astype(np.int32))
        ys.append(np.nan if r.y is None else float(np.asarray(r.y).reshape(-1)[0]))
        node_off.append(node_off[-1] + n)
        edge_off.append(edge_off[-1] + e)
        k0_off.append(k0_off[-1] + k0)
        p1_off.append(p1_off[-1] + prow.size)
        k1_off.append(k1_off[-1] + k1)

    cat = np.concatenate
    return PackedGraphs(
        n_feat=F,
        n_graphs=len(records),
        x=cat(xs),
        node_off=np.asarray(node_off, np.int64),
        edge_off=np.asarray(edge_off, np.int64),
        rowptr=cat(rps),
        col=cat(cols),
        eperm=cat(eperms),
        t_rowptr=cat(trps),
        t_col=cat(tcols),
        t_eid=cat(teids),
        transpose_aliased=bool(aliased),
        k0_off=np.asarray(k0_off, np.int64),
        m0_ptr=cat(m0ps),
        m0_idx=cat(m0is),
        cl0=cat(cl0s),
        p1_off=np.asarray(p1_off, np.int64),
        p1_rowptr=cat(p1rps),
        p1_col=cat(p1cs) if p1cs else np.zeros(0, np.int32),
        p1t_rowptr=cat(p1trps),
        p1t_col=cat(p1tcs) if p1tcs else np.zeros(0, np.int32),
        p1t_pid=cat(p1tps) if p1tps else np.zeros(0, np.int32),
        p1_ea=cat(p1eas) if has_ea else None,
        k1_off=np.asarray(k1_off, np.int64),
        m1_ptr=cat(m1ps),
        m1_idx=cat(m1is),
        cl1=cat(cl1s),
        y=np.asarray(ys, dtype=np.float32),
        edge_attr=cat(eas) if has_ea else None,
        names=[r.name for r in records],
        has_clusters=has_clusters,
    )


