"""TEST INFRASTRUCTURE ONLY (see ``oracle/__init__.py``).

Restatement of the MCL community detection the reference runs in
``Trainer._precluster`` (``deeprank2/trainer.py:319-348``) through
``community_detection`` (``deeprank2/utils/community_pooling.py:96-162``):

* networkx: ``nx.Graph`` over nodes ``0..N-1`` with one undirected, unweighted
  edge per ``edge_index`` column (duplicates merge), then
  ``nx.to_scipy_sparse_array(g).toarray()`` — a symmetric 0/1 adjacency;
* markov_clustering 0.0.6 (pinned in ``env/deeprank2_frozen.yml:164``; not
  installed in this image) ``run_mcl`` with its defaults — expansion 2,
  inflation 2, ``loop_value`` 1 (diagonal set to 1), 100 iterations, pruning
  threshold 1e-3 applied every iteration (column maxima kept), convergence by
  ``np.allclose(new, last)`` every iteration — and ``get_clusters``
  (attractors = non-zero diagonal, each attractor's row support is a cluster,
  unique clusters sorted lexicographically);
* the reference then writes ``index[list(c)] = ic`` for ic in that order.

Pinned by the stored ``clustering/mcl/depth_{0,1}`` of the reference's HDF5
fixtures (``tests/test_mcl.py``).
"""

from __future__ import annotations

import numpy as np


def adjacency(edge_index, num_nodes, edge_attr=None):
    """nx.Graph + add_edge in edge order (a repeated pair keeps the last
    weight, community_pooling.py:137-142) -> to_scipy_sparse_array().toarray()."""
    a = np.zeros((num_nodes, num_nodes), dtype=np.float64)
    ei = np.asarray(edge_index).reshape(2, -1)
    if edge_attr is None:
        a[ei[0], ei[1]] = 1.0
        a[ei[1], ei[0]] = 1.0
        return a
    for (i, j), w in zip(ei.T.tolist(), np.asarray(edge_attr, dtype=np.float64).reshape(-1).tolist()):
        a[i, j] = a[j, i] = w
    return a


def _normalize(m):
    """sklearn.preprocessing.normalize(m, norm='l1', axis=0): zero columns stay zero."""
    s = np.abs(m).sum(axis=0)
    s[s == 0.0] = 1.0
    return m / s


def _prune(m, threshold):
    pruned = m.copy()
    pruned[pruned < threshold] = 0.0
    cols = np.arange(m.shape[1])
    rows = m.argmax(axis=0)
    pruned[rows, cols] = m[rows, cols]
    return pruned


def run_mcl(matrix, expansion=2, inflation=2, loop_value=1, iterations=100, pruning_threshold=0.001):
    m = np.array(matrix, dtype=np.float64)
    if loop_value > 0:
        np.fill_diagonal(m, loop_value)
    m = _normalize(m)
    for _ in range(iterations):
        last = m.copy()
        m = np.linalg.matrix_power(m, expansion)
        m = _normalize(np.power(m, inflation))
        if pruning_threshold > 0:
            m = _prune(m, pruning_threshold)
        if np.allclose(m, last):
            break
    return m


def get_clusters(m):
    attractors = m.diagonal().nonzero()[0]
    clusters = {tuple(m[a].nonzero()[0].tolist()) for a in attractors}
    return sorted(clusters)


def mcl_community_detection(edge_index, num_nodes, edge_attr=None):
    """community_pooling.py:150-162 (method='mcl')."""
    clusters = get_clusters(run_mcl(adjacency(edge_index, num_nodes, edge_attr)))
    index = np.zeros(num_nodes, dtype=np.int64)
    for ic, c in enumerate(clusters):
        index[list(c)] = ic
    return index
