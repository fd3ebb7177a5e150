"""Helpers shared by the test modules (golden arrays -> inputs, state dicts)."""

from __future__ import annotations

import numpy as np
import torch

from oracle import pyg_ops as P


def golden_batch(z):
    """Rebuild the collated PyG-style batch stored by tests/golden/make_golden.py."""
    b = P.Batch()
    for k in ("x", "edge_index", "edge_attr", "batch", "cluster0", "cluster1", "y", "pos", "ptr"):
        key = "in/" + k
        if key in z:
            arr = z[key]
            t = torch.from_numpy(np.array(arr))
            b.__dict__[k] = t
    return b


def golden_state_dict(z):
    return {k[len("param/"):]: torch.from_numpy(np.array(v)) for k, v in z.items() if k.startswith("param/")}


def golden_grads(z):
    return {k[len("grad/"):]: np.array(v) for k, v in z.items() if k.startswith("grad/")}


def fixed_dropout(mask):
    def _drop(x, p, training):
        return x * mask / (1.0 - p) if training else x

    return _drop


def assert_grad_close(actual, ref, rtol=1e-4, ntol=1e-6, err_msg=""):
    """Gradient parity: elementwise rtol plus a normwise floor ntol*max|ref|.

    fp32 reassociation (the MI355X path aggregates A·X before the GEMM; the
    reference multiplies per edge, then scatter-adds) leaves absolute errors
    that scale with the tensor's largest entries (~1e3 on the 1ATN fixture),
    so tiny entries of a large gradient need the normwise floor."""
    ref = np.asarray(ref)
    fin = np.abs(ref[np.isfinite(ref)])
    scale = float(fin.max()) if fin.size else 0.0  # NaN entries must match NaN (assert_allclose equal_nan)
    np.testing.assert_allclose(np.asarray(actual), ref, rtol=rtol, atol=max(1e-6, ntol * scale), err_msg=err_msg)


def golden_graphs(z):
    """Per-graph (local edge_index, num_nodes, cluster0, cluster1) of a stored
    collated batch (``in/ptr`` node offsets; cluster1 has one entry per
    depth-0 cluster of each graph)."""
    ptr, ei, c0, c1 = (np.asarray(z[f"in/{k}"]) for k in ("ptr", "edge_index", "cluster0", "cluster1"))
    out, k1 = [], 0
    for g in range(ptr.size - 1):
        lo, hi = int(ptr[g]), int(ptr[g + 1])
        m = (ei[0] >= lo) & (ei[0] < hi)
        a = c0[lo:hi]
        k = int(a.max()) + 1 if a.size else 0
        out.append((ei[:, m] - lo, hi - lo, a, c1[k1 : k1 + k]))
        k1 += k
    assert k1 == c1.size
    return out
