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
