"""Batched MCL community detection on the GPU (``dr_mcl`` / ``dr_mcl_assign``).

Replaces what ``Trainer._precluster`` (``deeprank2/trainer.py:319-348``) does
graph by graph through networkx + markov_clustering
(``deeprank2/utils/community_pooling.py:96-162``): depth 0 on each graph,
then depth 1 on the graph pooled by the depth-0 clusters
(``community_pooling`` -> PyG ``pool_edge``: relabelled to consecutive ids,
self loops dropped).  All graphs of a chunk run in one launch (one workgroup
per graph, float64); the host keeps only the integer bookkeeping (CSR build,
``get_clusters`` ordering).

Louvain (``python-louvain`` ``best_partition``, randomised) is not provided.
"""

from __future__ import annotations

import ctypes

import numpy as np
import torch

from deeprank2_amd import _lib

MAX_ITER = 100  # markov_clustering.run_mcl defaults
PRUNING_THRESHOLD = 1e-3
WORKSPACE_BUDGET = 4 << 30  # bytes of fp64 workspace per launch (chunks above that)


def _symmetric_weighted(src, dst, w):
    """networkx Graph.add_edge(i, j, weight=w) in edge order: one undirected
    edge per pair, the last weight wins; returned as both directions."""
    lo, hi = np.minimum(src, dst), np.maximum(src, dst)
    key = lo * (int(hi.max(initial=0)) + 1) + hi
    last = {}
    for k, v in zip(key.tolist(), np.asarray(w, dtype=np.float64).tolist()):
        last[k] = v
    keys = np.fromiter(last.keys(), dtype=np.int64, count=len(last))
    vals = np.fromiter(last.values(), dtype=np.float64, count=len(last))
    m = int(hi.max(initial=0)) + 1
    a, b = keys // m, keys % m
    return np.concatenate([a, b]), np.concatenate([b, a]), np.concatenate([vals, vals])


def _layout(graphs, weights):
    """Local CSR of every graph: rowptr (graph g's N+1 entries at node_off[g] + g),
    col / weight at edge_off[g]."""
    n = np.array([g[1] for g in graphs], dtype=np.int64)
    node_off = np.zeros(len(graphs) + 1, dtype=np.int64)
    np.cumsum(n, out=node_off[1:])
    srcs, dsts, ws = [], [], []
    for k, (ei, nn) in enumerate(graphs):
        ei = np.asarray(ei, dtype=np.int64).reshape(2, -1)
        if ei.size and (ei.min() < 0 or ei.max() >= nn):
            msg = f"graph {k}: edge_index refers to nodes outside 0..{nn - 1}"
            raise ValueError(msg)
        s, d = ei[0], ei[1]
        w = None
        if weights is not None:
            s, d, w = _symmetric_weighted(s, d, np.asarray(weights[k]).reshape(-1))
            ws.append(w)
        srcs.append(s + node_off[k])
        dsts.append(d)
    gsrc = np.concatenate(srcs) if srcs else np.zeros(0, np.int64)
    dst = np.concatenate(dsts) if dsts else np.zeros(0, np.int64)
    order = np.argsort(gsrc, kind="stable")
    col = dst[order].astype(np.int32)
    weight = np.concatenate(ws)[order] if weights is not None and ws else None
    tot = int(node_off[-1])
    grp = np.zeros(tot + 1, dtype=np.int64)
    np.cumsum(np.bincount(gsrc, minlength=tot), out=grp[1:])
    edge_off = grp[node_off]
    gid = np.repeat(np.arange(len(graphs)), n + 1)
    pos = np.arange(tot + len(graphs)) - (node_off[gid] + gid)
    rowptr = (grp[node_off[gid] + pos] - edge_off[gid]).astype(np.int32)
    return n, node_off, rowptr, edge_off, col, weight


def mcl_clusters(graphs, device=None, weights=None, max_iter=MAX_ITER, pruning_threshold=PRUNING_THRESHOLD, return_iters=False):
    """Cluster ids (int64 numpy, one array per graph) of ``graphs`` = list of
    ``(edge_index [2,E], num_nodes)``; ``weights`` = optional per-graph edge
    weights (``community_detection(edge_attr=...)``)."""
    device = torch.device("cuda", torch.cuda.current_device()) if device is None else torch.device(device)
    if device.type != "cuda":
        msg = "MCL runs on the MI355X only (no CPU fallback by design)"
        raise RuntimeError(msg)
    lib = _lib.load()
    out, iters_out = [None] * len(graphs), [0] * len(graphs)
    # chunk by workspace size
    chunks, cur, cur_bytes = [], [], 0
    for k, (_, nn) in enumerate(graphs):
        b = 8 * int(lib.dr_mcl_workspace_doubles(int(nn)))
        if cur and cur_bytes + b > WORKSPACE_BUDGET:
            chunks.append(cur)
            cur, cur_bytes = [], 0
        cur.append(k)
        cur_bytes += b
    if cur:
        chunks.append(cur)
    for ch in chunks:
        sub = [graphs[k] for k in ch]
        n, node_off, rowptr, edge_off, col, weight = _layout(sub, None if weights is None else [weights[k] for k in ch])
        wsz = np.array([lib.dr_mcl_workspace_doubles(int(v)) for v in n], dtype=np.int64)
        ws_off = np.zeros(len(sub) + 1, dtype=np.int64)
        np.cumsum(wsz, out=ws_off[1:])
        pat_off = np.zeros(len(sub) + 1, dtype=np.int64)
        np.cumsum(n * n, out=pat_off[1:])
        dev = {k: torch.from_numpy(v).to(device) for k, v in (("node_off", node_off), ("rowptr", rowptr), ("edge_off", edge_off), ("col", col), ("ws_off", ws_off), ("pat_off", pat_off))}
        dev["weight"] = None if weight is None else torch.from_numpy(weight).to(device)
        ws = torch.empty(int(ws_off[-1]), dtype=torch.float64, device=device)
        pattern = torch.empty(max(1, int(pat_off[-1])), dtype=torch.uint8, device=device)
        iters = torch.zeros(len(sub), dtype=torch.int32, device=device)
        if dev["col"].numel() == 0:
            dev["col"] = torch.zeros(1, dtype=torch.int32, device=device)
        gc = _lib.MclGraphsC(
            node_off=dev["node_off"].data_ptr(), rowptr=dev["rowptr"].data_ptr(), edge_off=dev["edge_off"].data_ptr(),
            col=dev["col"].data_ptr(), weight=None if dev["weight"] is None else dev["weight"].data_ptr(),
            ws_off=dev["ws_off"].data_ptr(), ws=ws.data_ptr(), pat_off=dev["pat_off"].data_ptr(), pattern=pattern.data_ptr(), iters=iters.data_ptr(),
        )
        with torch.cuda.device(device):
            _lib.check(lib.dr_mcl(ctypes.byref(gc), len(sub), int(max_iter), float(pruning_threshold), _lib.stream_ptr(device)), "dr_mcl")
            pat = pattern.cpu().numpy()
        cl = np.zeros(int(node_off[-1]), dtype=np.int32)
        _lib.check(lib.dr_mcl_assign(pat.ctypes.data, pat_off.ctypes.data, node_off.ctypes.data, len(sub), cl.ctypes.data, None), "dr_mcl_assign")
        it = iters.cpu().numpy()
        for j, k in enumerate(ch):
            out[k] = cl[node_off[j] : node_off[j + 1]].astype(np.int64)
            iters_out[k] = int(it[j])
        del ws
    return (out, iters_out) if return_iters else out


def pooled_graph(cluster, edge_index):
    """``community_pooling(cluster, data)``'s graph (consecutive_cluster +
    pool_edge): (edge_index [2,E'], num_clusters)."""
    uniq, dense = np.unique(np.asarray(cluster, dtype=np.int64), return_inverse=True)
    ei = np.asarray(edge_index, dtype=np.int64).reshape(2, -1)
    r, c = dense[ei[0]], dense[ei[1]]
    keep = r != c
    k = max(1, uniq.size)
    key = np.unique(r[keep] * k + c[keep])
    return np.stack([key // k, key % k]), int(uniq.size)


def precluster_graphs(graphs, device=None):
    """(depth_0, depth_1) per graph, as ``Trainer._precluster`` computes them."""
    c0 = mcl_clusters(graphs, device)
    pooled = [pooled_graph(c, ei) for c, (ei, _) in zip(c0, graphs)]
    c1 = mcl_clusters(pooled, device)
    return c0, c1
