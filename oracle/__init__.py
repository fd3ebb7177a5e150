"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the DeepRank2 GNN hot path.

Nothing in the product (``deeprank-gnn-2_amd/deeprank2_amd``) imports, links or
executes anything from this package.  Only ``tests/``, ``__graft_entry__.smoke()``
and the ``cpu_baseline`` leg of ``bench.py`` may use it, and only as the checker
or as the timed CPU baseline, never as the thing measured on the GPU.

Contents
--------
``pyg_ops``    torch-CPU restatement of the third-party ops the reference calls
               (torch_scatter 2.1.2 ``scatter_sum/mean/max``; PyG 2.4.0
               ``consecutive_cluster``, ``pool_edge``, ``pool_batch``,
               ``max_pool_x``, ``inits.uniform``, ``Data``/``Batch``).
               These libraries are not installed anywhere in this image, so
               their semantics are restated from the pinned versions'
               documented behaviour: parity at that boundary is UNPINNED
               (SURVEY.md §8(c)).
``gnn_ref``    op-for-op torch-CPU restatement of ``deeprank2/neuralnets/gnn``
               (GINet, FoutNet, VanillaNetwork) and
               ``deeprank2/utils/community_pooling.py``.
``data_ref``   restatement of ``GraphDataset.load_one_graph`` + PyG collate over
               the ``.npz`` dump of the HDF5 fixtures.
``mcl_ref``    numpy restatement of networkx's adjacency + markov_clustering
               0.0.6 ``run_mcl`` / ``get_clusters`` (``Trainer._precluster``).

(The seeded synthetic graph generator of SURVEY.md §8(d) is not oracle code: it
lives in the package, ``deeprank2_amd.utils.synthetic``.)

Pinning: ``gnn_ref`` and ``pyg_ops`` are checked in ``tests/test_oracle.py``
against golden vectors produced by importing the *reference's own*
``deeprank2.neuralnets.gnn`` modules (``tests/golden/make_golden.py``).  The
golden run uses stand-ins for PyG/torch_scatter (``tests/golden/refshim``) that
forward to ``pyg_ops``, so what is pinned is the deeprank2 code; the PyG /
torch_scatter semantics themselves remain unpinned (no fixture in the reference
asserts them).
"""
